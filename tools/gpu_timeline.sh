#!/bin/bash
# Kernel timeline of the headline bench (768 chains, default stream groups): one kernel trace,
# kept, summarised by tools/timeline.py.  usage: bash tools/gpu_timeline.sh <tag> [bench args]
tag=${1:-tl}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_$tag -o run -- python bench.py --no-cpu --no-single --no-match --no-sequence --steps 6 --warmup 3 "$@" > gpurun_out/tl_$tag.log 2>&1 || exit $?
python tools/timeline.py gpurun_out/tl_$tag > gpurun_out/tl_$tag.txt
rm -f gpurun_out/tl_$tag/*kernel_trace.csv.bak
head -120 gpurun_out/tl_$tag.txt
