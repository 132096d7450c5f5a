#!/bin/bash
# round-5: matcher merge + fixup fused into k_bf_i8's tail -- matcher tests, C3 / C5 matcher A/B
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
BASE=$PWD/monocular_visual_odometry_va4mr_amd/_build/libvo_base.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bootstrap.py tests/test_gpu_configs.py tests/test_gpu_streams.py > gpurun_out/r5r_tests.log 2>&1 || { tail -30 gpurun_out/r5r_tests.log; exit 1; }
tail -1 gpurun_out/r5r_tests.log
for i in 1 2; do
  timeout -k 10 300 python -u tools/c3_only.py 1 | sed 's/^/new  /' || exit 1
  VO_HIP_LIB=$BASE timeout -k 10 300 python -u tools/c3_only.py 1 | sed 's/^/base /' || exit 1
done
