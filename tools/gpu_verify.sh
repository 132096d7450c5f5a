#!/bin/bash
# One GPU verification call: parity tests, default bench line, rocprofv3 kernel stats.
# usage: bash tools/gpu_verify.sh <tag>
tag=${1:-v}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_$tag.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --stages > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || exit $?
cat gpurun_out/bench_$tag.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --kernel-include-regex "::k_" --output-format csv -d gpurun_out/prof_$tag -o run -- python bench.py --no-cpu --no-single --steps 20 > gpurun_out/prof_$tag.log 2>&1 || exit $?
rm -f gpurun_out/prof_$tag/*kernel_trace.csv
ls gpurun_out/prof_$tag
