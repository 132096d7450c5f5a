#!/bin/bash
# triangulation in three passes + single-scan PnP apply: GPU tests, PnP phase profile,
# single-chain latency.  usage: gpu_tri.sh <tag>
tag=${1:-a}
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tri_${tag}_pytest.txt 2>&1 || { tail -30 gpurun_out/tri_${tag}_pytest.txt; exit 1; }
tail -3 gpurun_out/tri_${tag}_pytest.txt
timeout -k 10 120 python -u tools/pnp_prof.py 80 > gpurun_out/tri_${tag}_pnp.log 2>&1 || exit 1
tail -4 gpurun_out/tri_${tag}_pnp.log
for v in 0 1 0 1; do echo "VO_GFTT_LATE=$v"; VO_GFTT_LATE=$v timeout -k 10 200 python -u tools/single_prof.py 200 2>&1 | grep frames; done
for v in 0 1; do echo "bench VO_GFTT_LATE=$v"; VO_GFTT_LATE=$v timeout -k 10 300 python -u bench.py --no-cpu --no-single --no-match --no-sequence --steps 30 --warmup 5 2>&1 | tail -1 | cut -c1-400; done
