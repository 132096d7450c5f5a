#!/bin/bash
# round-5 late: kernel trace of rank 0's slice of the 8-GPU sequence plan (24 shards, overlap 15)
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sl8b -o run -- python tools/slice_sweep.py 8:24:15 --reps 3 > gpurun_out/sl8b.log 2>&1 || { tail -5 gpurun_out/sl8b.log; exit 1; }
python tools/trace_by_grid.py gpurun_out/sl8b gpurun_out/sl8b/by_grid.csv
python tools/timeline.py gpurun_out/sl8b 400 > gpurun_out/sl8b_timeline.txt
rm -f gpurun_out/sl8b/*kernel_trace.csv
head -25 gpurun_out/sl8b/by_grid.csv; cat gpurun_out/sl8b.log | tail -3
