#!/bin/bash
# RANSAC scoring batches + hypotheses over all waves: GPU tests, PnP phase profile, single
# chain, headline.  usage: gpu_ransac.sh <tag>
tag=${1:-a}
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ransac_${tag}_pytest.txt 2>&1 || { tail -30 gpurun_out/ransac_${tag}_pytest.txt; exit 1; }
tail -3 gpurun_out/ransac_${tag}_pytest.txt
timeout -k 10 120 python -u tools/pnp_prof.py 80 > gpurun_out/ransac_${tag}_pnp.log 2>&1 || exit 1
tail -4 gpurun_out/ransac_${tag}_pnp.log
for v in 1 2 3; do timeout -k 10 200 python -u tools/single_prof.py 200 2>&1 | grep frames; done
for v in 1 2; do timeout -k 10 300 python -u bench.py --no-cpu --no-single --no-match --no-sequence --steps 30 --warmup 5 2>&1 | tail -1 | cut -c1-300; done
