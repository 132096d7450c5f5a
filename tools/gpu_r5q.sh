#!/bin/bash
# round-5: C5 step kernels alone (128 chains, one group, every stage on one stream) and the default C5 leg traced
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
VO_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5solo -o run -- python tools/c5_only.py 128 1 > gpurun_out/c5solo.log 2>&1 || { tail -5 gpurun_out/c5solo.log; exit 1; }
python tools/trace_by_grid.py gpurun_out/c5solo gpurun_out/c5solo/by_grid.csv && rm -f gpurun_out/c5solo/*kernel_trace.csv
grep -v "sift\|blur\|extrema\|upsample\|bf_\|essential\|recover\|nn_down" gpurun_out/c5solo/by_grid.csv | head -14
tail -1 gpurun_out/c5solo.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c5tl -o run -- python tools/c5_only.py 256 2 > gpurun_out/c5tl.log 2>&1 || { tail -5 gpurun_out/c5tl.log; exit 1; }
python tools/timeline.py gpurun_out/c5tl 60 > gpurun_out/c5_timeline.txt && rm -f gpurun_out/c5tl/*kernel_trace.csv
cat gpurun_out/c5_timeline.txt; tail -1 gpurun_out/c5tl.log
