#!/bin/bash
# round-5: kernel trace of rank 0's slice of the 8-GPU sequence plan (24 shards, overlap 15)
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sl8 -o run -- python tools/slice_sweep.py 8:24:15 --reps 3 > gpurun_out/sl8.log 2>&1 || { tail -5 gpurun_out/sl8.log; exit 1; }
python tools/trace_by_grid.py gpurun_out/sl8 gpurun_out/sl8/by_grid.csv
python tools/timeline.py gpurun_out/sl8 400 > gpurun_out/sl8_timeline.txt
rm -f gpurun_out/sl8/*kernel_trace.csv
head -25 gpurun_out/sl8/by_grid.csv; cat gpurun_out/sl8.log | tail -3
