#!/bin/bash
# C5 (1920x1080, 8,192 corners): chains x groups sweep, then a kernel trace of the default leg
# (per-launch-shape summary, the raw trace deleted)
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/c5_only.py 256 2 256 1 128 1 128 2 384 3 512 2 > gpurun_out/c5_sweep.jsonl 2> gpurun_out/c5_sweep.err || { tail -5 gpurun_out/c5_sweep.err; exit 1; }
cat gpurun_out/c5_sweep.jsonl
rm -rf gpurun_out/c5prof
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5prof -o c5 -- python3 tools/c5_only.py 256 2 > gpurun_out/c5prof.log 2>&1 || { tail -5 gpurun_out/c5prof.log; exit 1; }
python3 tools/trace_by_grid.py gpurun_out/c5prof gpurun_out/c5prof_by_grid.csv && head -16 gpurun_out/c5prof_by_grid.csv
python3 tools/timeline.py gpurun_out/c5prof 300 > gpurun_out/c5prof_timeline.txt
rm -rf gpurun_out/c5prof
