#!/bin/bash
# GPU session: parity tests + bench sweep over chains per GPU.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for c in 16 64 128; do
  timeout -k 10 400 python bench.py --chains $c --steps 20 --warmup 5 --no-cpu --stages > gpurun_out/bench_c$c.json 2> gpurun_out/bench_c$c.err || exit $?
  cat gpurun_out/bench_c$c.json
done
