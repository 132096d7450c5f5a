#!/bin/bash
# LK parity tests with an alternative build, then the alternating headline A/B (gpu_libab.sh).
# usage: bash tools/gpu_lkab.sh <tag> <alt.so> [reps]
tag=$1; alt=$2; reps=${3:-2}
mkdir -p gpurun_out
export TMPDIR=/tmp
VO_HIP_LIB=$PWD/$alt timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    -k "lk or step_parity" > gpurun_out/lkab_${tag}_t.log 2>&1 || { tail -20 gpurun_out/lkab_${tag}_t.log; exit 1; }
tail -1 gpurun_out/lkab_${tag}_t.log
bash tools/gpu_libab.sh $PWD/$alt $reps
