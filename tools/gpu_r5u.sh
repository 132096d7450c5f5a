#!/bin/bash
# round-5: one chain (drop-in mode) kernel timeline
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sc -o run -- python tools/single_prof.py 100 > gpurun_out/sc.log 2>&1 || { tail -5 gpurun_out/sc.log; exit 1; }
python tools/timeline.py gpurun_out/sc 60 > gpurun_out/sc_timeline.txt && python tools/trace_by_grid.py gpurun_out/sc gpurun_out/sc/by_grid.csv && rm -f gpurun_out/sc/*kernel_trace.csv
cat gpurun_out/sc_timeline.txt; grep frames_per_s gpurun_out/sc.log
