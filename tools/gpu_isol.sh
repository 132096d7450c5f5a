#!/bin/bash
# Isolated per-kernel times of the step (every stage on one stream, one group of 384 chains):
# kernel trace -> per-grid summary.  usage: bash tools/gpu_isol.sh <tag> [bench args]
tag=${1:-is}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp VO_ONE_STREAM=1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/is_$tag -o run -- python bench.py --no-cpu --no-single --no-match --no-sequence --groups 1 --chains 384 --steps 10 --warmup 3 "$@" > gpurun_out/is_$tag.log 2>&1 || exit $?
python tools/trace_by_grid.py gpurun_out/is_$tag gpurun_out/is_$tag/by_grid.csv
rm -f gpurun_out/is_$tag/*kernel_trace.csv
head -16 gpurun_out/is_$tag/by_grid.csv
