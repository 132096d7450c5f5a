#!/bin/bash
# Kernel trace of the C5 (1920x1080, 64 chains) leg alone -> per-grid summary.
tag=${1:-c5}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c5_$tag -o run -- python tools/c5_only.py > gpurun_out/c5_$tag.log 2>&1 || exit $?
python tools/trace_by_grid.py gpurun_out/c5_$tag gpurun_out/c5_$tag/by_grid.csv
rm -f gpurun_out/c5_$tag/*kernel_trace.csv
head -14 gpurun_out/c5_$tag/by_grid.csv
tail -1 gpurun_out/c5_$tag.log | cut -c1-600
