#!/bin/bash
# round-4 probe 4: kernel trace of the 64-chain 2-group sequence job (summaries only: the raw
# trace is deleted, gpurun_out must stay under 64 MiB); then the headline A/B (probe 3)
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
rm -rf gpurun_out/seqprof
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/seqprof -o seq -- python3 tools/seq_sweep.py 64 --groups 2 --reps 2 > gpurun_out/seqprof.log 2>&1 || { tail -5 gpurun_out/seqprof.log; exit 1; }
python3 tools/trace_by_grid.py gpurun_out/seqprof gpurun_out/seqprof_by_grid.csv && head -25 gpurun_out/seqprof_by_grid.csv
python3 tools/timeline.py gpurun_out/seqprof 400 > gpurun_out/seqprof_timeline.txt
find gpurun_out/seqprof -name "*stats.csv" -exec cp {} gpurun_out/seqprof_kernel_stats.csv \;
rm -rf gpurun_out/seqprof
bash tools/gpu_r4probe3.sh
