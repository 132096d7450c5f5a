#!/bin/bash
# pyramid levels 0 and 1 in one launch (k_pyr01, default at <= 64 chains): the GPU suite, then
# alternating A/B against five launches (VO_PYR01=0) on the single chain and the sequence job
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
[ "$1" = notests ] || bash tools/gpu_r4tests.sh || exit 1
for rep in 1 2; do
  for p in 1 0; do
    VO_PYR01=$p timeout -k 10 120 python -u tools/single_prof.py 100 2>/dev/null | sed "s/^/pyr01=$p single /" || exit 1
    VO_PYR01=$p timeout -k 10 300 python -u tools/seq_sweep.py --groups 2 --reps 2 --no-boot-sync 64 > gpurun_out/p01.jsonl 2> gpurun_out/p01.err || { tail -3 gpurun_out/p01.err; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/p01.jsonl'):
    d=json.loads(l); print('pyr01=$p seq', d['sequence_frames_per_s'], d['wall_s'], d['bootstrap_s'], d['ms_per_step'], d['shards_ok'], (d.get('vs_reference') or {}).get('shards_identical'))"
  done
done
