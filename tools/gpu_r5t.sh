#!/bin/bash
# round-5: deeper row prefetch in k_pyr_rows -- pyramid tests, pyramid alone, headline A/B vs libvo_base.so
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
BASE=$PWD/monocular_visual_odometry_va4mr_amd/_build/libvo_base.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "pyramid or lk or step" > gpurun_out/r5t_tests.log 2>&1 || { tail -30 gpurun_out/r5t_tests.log; exit 1; }
tail -1 gpurun_out/r5t_tests.log
for i in 1 2; do
  timeout -k 10 200 python tools/pyr_bench.py 384 768 | sed "s/^/new  /" || exit 1
  VO_HIP_LIB=$BASE timeout -k 10 200 python tools/pyr_bench.py 384 768 | sed "s/^/base /" || exit 1
done
bash tools/gpu_ab.sh r5t 2
