#!/bin/bash
# LK change A/B in one GPU call: the LK / step bit-exact tests on the default build, then the
# headline bench alternating the default build with a saved one.
# usage: bash tools/gpu_lkab.sh <tag> <alt.so> [reps]
tag=${1:-ab}; alt=$2; n=${3:-2}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/lkab_$tag.log 2>&1 || { tail -30 gpurun_out/lkab_$tag.log; exit 1; }
tail -1 gpurun_out/lkab_$tag.log
bash tools/gpu_libab.sh $alt $n
