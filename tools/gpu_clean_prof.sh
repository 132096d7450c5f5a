#!/bin/bash
# Uncontended per-kernel profile: one engine group, every stage on one stream, so kernel
# durations are not inflated by concurrent streams.  Kernel stats + FETCH/WRITE passes.
# usage: bash tools/gpu_clean_prof.sh <tag> [bench args...]
tag=${1:-c}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp VO_ONE_STREAM=1
A="--no-cpu --no-single --groups 1 --chains 192 --steps 10 --warmup 3 $@"
R="--kernel-include-regex ::k_ --output-format csv"
timeout -k 10 300 python bench.py --stages $A > gpurun_out/cbench_$tag.json 2> gpurun_out/cbench_$tag.err || exit $?
cat gpurun_out/cbench_$tag.json; tail -1 gpurun_out/cbench_$tag.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats $R -d gpurun_out/cprof_$tag -o run -- python bench.py $A > gpurun_out/cprof_$tag.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE $R -d gpurun_out/cfetch_$tag -o run -- python bench.py $A > gpurun_out/cfetch_$tag.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE $R -d gpurun_out/cwrite_$tag -o run -- python bench.py $A > gpurun_out/cwrite_$tag.log 2>&1 || exit $?
rm -f gpurun_out/cprof_$tag/*kernel_trace.csv
du -sh gpurun_out/c*_$tag
