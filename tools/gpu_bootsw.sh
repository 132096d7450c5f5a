#!/bin/bash
# bootstrap of 768 chains: essential-RANSAC variants (VO_ESS_VARIANT bit 0: 2 waves/SIMD build when
# chains > CUs, bit 1: five-point solves spread over four waves) and the SIFT workspace budget
# per engine (VO_SIFT_BATCH_BYTES).  usage: gpu_bootsw.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for v in 0 3; do
  VO_ESS_VARIANT=$v timeout -k 10 400 python -u -m pytest tests/test_gpu_bootstrap.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -1
done
run() { timeout -k 10 200 python -u bench.py --no-cpu --no-single --no-match --no-sequence --steps 3 --warmup 1 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['bootstrap_s'], d['bootstrap_workspace_alloc_s'], d['value'], d['chains_ok'])"; }
for r in 1 2; do
  for v in 0 1 2 3; do echo "variant $v 24GB: $(VO_ESS_VARIANT=$v run)"; done
  for gb in 64 110; do echo "variant 0 ${gb}GB: $(VO_SIFT_BATCH_BYTES=$((gb << 30)) run)"; done
done
