#!/bin/bash
# parity tests (optionally a -k filter) then the uncontended bench line
# usage: bash tools/gpu_quick.sh <tag> [pytest -k expr]
tag=${1:-q}; k=${2:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$k" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$k" > gpurun_out/pytest_$tag.log 2>&1
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
fi
rc=$?
tail -4 gpurun_out/pytest_$tag.log
[ $rc -ne 0 ] && exit $rc
VO_ONE_STREAM=1 timeout -k 10 300 python bench.py --stages --no-cpu --no-single --groups 1 --chains 192 --steps 10 --warmup 3 > gpurun_out/cbench_$tag.json 2> gpurun_out/cbench_$tag.err || exit $?
tail -1 gpurun_out/cbench_$tag.err
timeout -k 10 300 python bench.py --no-cpu --no-single > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || exit $?
cat gpurun_out/bench_$tag.json
