#!/bin/bash
# GPU check: parity tests, then bench + rocprofv3 stats (k_* kernels only).
# usage: bash tools/gpu_check.sh <tag> [bench args...]
tag=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_$tag.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_$tag.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --no-cpu --stages "$@" > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || exit $?
cat gpurun_out/bench_$tag.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --kernel-include-regex "::k_" --output-format csv -d gpurun_out/prof_$tag -o run -- python bench.py --no-cpu --no-single "$@" > gpurun_out/prof_$tag.log 2>&1 || exit $?
rm -f gpurun_out/prof_$tag/*kernel_trace.csv
exit $rc
