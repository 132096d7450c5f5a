#!/bin/bash
# one-launch pyramid for small batches: GPU tests, PnP phase profile, single-chain A/B
# (VO_PYR_ONE=1 default vs 0 = per-level launches).  usage: gpu_pyr1.sh <tag>
tag=${1:-a}
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
L=gpurun_out/pyr1_${tag}.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pyr1_${tag}_pytest.txt 2>&1 || { tail -30 gpurun_out/pyr1_${tag}_pytest.txt; exit 1; }
tail -3 gpurun_out/pyr1_${tag}_pytest.txt
timeout -k 10 120 python -u tools/pnp_prof.py 80 > gpurun_out/pyr1_${tag}_pnp.log 2>&1 || exit 1
tail -2 gpurun_out/pyr1_${tag}_pnp.log
for v in 1 0 1 0; do
  echo "VO_PYR_ONE=$v" >> $L
  VO_PYR_ONE=$v timeout -k 10 200 python -u tools/single_prof.py 200 >> $L 2>&1 || exit 1
done
cat $L
