#!/bin/bash
# LK staging change: GPU tests, LK part timings, headline bench (short)
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash tools/gpu_r4tests.sh || exit 1
bash tools/lk_parts.sh || exit 1
for r in 1 2; do
timeout -k 10 200 python -u bench.py --no-cpu --no-single --no-match --no-sequence --steps 20 --warmup 5 > gpurun_out/lkb.json 2> gpurun_out/lkb.err || { tail -5 gpurun_out/lkb.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/lkb.json').read().splitlines()[-1])
print('headline', d['value'], d['ms_per_step'], d['chains_ok'], d['stages_ms'])"
done
