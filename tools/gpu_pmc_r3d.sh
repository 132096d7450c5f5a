#!/bin/bash
# PMC passes of the headline (FETCH/WRITE, k_lk_w SQ) and the single-chain legs after the
# headline with the high-priority side stream for small batches.  usage: gpu_pmc_r3d.sh <tag>
tag=${1:-r3d}
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pmc_${tag}_pytest.txt 2>&1 || { tail -20 gpurun_out/pmc_${tag}_pytest.txt; exit 1; }
tail -1 gpurun_out/pmc_${tag}_pytest.txt
timeout -k 10 300 python bench.py --no-cpu --no-match > gpurun_out/prio_$tag.json 2> gpurun_out/prio_$tag.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/prio_$tag.json').read().splitlines()[-1]); print(d['value'], d['single_chain'])"
bash tools/gpu_prof_r3.sh pmc $tag
