#!/bin/bash
# status filtering fused into the PnP launch (default) vs the separate compaction launch
# (VO_COMPACT_IN_TRACK=1):
# the whole GPU suite, then alternating A/B on the sequence job, the single chain and the headline
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
[ "$1" = notests ] || bash tools/gpu_r4tests.sh || exit 1
for rep in 1 2; do
  for cfg in "X=0" "VO_COMPACT_IN_TRACK=1"; do
    env $cfg timeout -k 10 300 python -u tools/seq_sweep.py --groups 2 --reps 2 --no-boot-sync 64 > gpurun_out/fz_seq.jsonl 2> gpurun_out/fz.err || { tail -5 gpurun_out/fz.err; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/fz_seq.jsonl'):
    d=json.loads(l); print('$cfg seq', d['sequence_frames_per_s'], d['wall_s'], d['ms_per_step'], d['shards_ok'], (d.get('vs_reference') or {}).get('shards_identical'))"
  done
  for c in 0 1; do
    VO_COMPACT_IN_TRACK=$c timeout -k 10 300 python -u bench.py --no-cpu --no-match --no-sequence --steps 20 --warmup 5 > gpurun_out/fz_bench.json 2>> gpurun_out/fz.err || { tail -5 gpurun_out/fz.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/fz_bench.json').read().splitlines()[-1])
print('compact_in_track=$c headline', d['value'], d['ms_per_step'], d['chains_ok'], 'single', d['single_chain']['frames_per_s'], d['single_chain']['graph_frames_per_s'], d['single_chain']['graph_identical'])"
  done
done
