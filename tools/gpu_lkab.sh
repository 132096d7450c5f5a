#!/bin/bash
# LK A/B: the LK parity tests on the default kernel, then the headline bench (no side legs)
# alternating VO_LK_HALF=1 (k_lk_h, two points per wave) and 0 (k_lk_w).
# usage: bash tools/gpu_lkab.sh <tag> [reps]
tag=${1:-ab}
reps=${2:-2}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "lk or step_parity or full_sequence or sharded_sequence or full_pipeline" > gpurun_out/lkab_pytest_$tag.log 2>&1
rc=$?
tail -3 gpurun_out/lkab_pytest_$tag.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/lkab_pytest_$tag.log | head -20; exit $rc; }
A="--no-single --no-match --no-sequence --no-cpu --stages"
for i in $(seq 1 $reps); do
  for h in 1 0; do
    VO_LK_HALF=$h timeout -k 10 300 python bench.py $A > gpurun_out/lkab_${tag}_h${h}_$i.json 2> gpurun_out/lkab_${tag}_h${h}_$i.err || { tail -5 gpurun_out/lkab_${tag}_h${h}_$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('half', sys.argv[2], d['value'], d['ms_per_step'], d['stages_ms'])" gpurun_out/lkab_${tag}_h${h}_$i.json $h
  done
done
