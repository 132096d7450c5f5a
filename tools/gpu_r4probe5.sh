#!/bin/bash
# round-4 probe 5: the 64-chain sequence job under launch-shape options (LK blocks per chain,
# PnP build, latency stream priority); pre-gathered step frames
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 200 python -u tools/seq_sweep.py 64 --groups 2 --reps 3 > gpurun_out/p5.jsonl 2> gpurun_out/p5.err || { tail -5 gpurun_out/p5.err; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/p5.jsonl'):
    d=json.loads(l); print('$*', d['sequence_frames_per_s'], d['wall_s'], d['bootstrap_s'], d['ms_per_step'], d['shards_ok'], (d.get('vs_reference') or {}).get('shards_identical'))"
}
run X=0
run VO_LK_NB=512
run VO_LK_NB=256
run VO_PNP_TRI_WPE=2
run VO_PRIO_LATENCY=1
run VO_LK_NB=512 VO_PNP_TRI_WPE=2
run VO_LK_NB=256 VO_PNP_TRI_WPE=2 VO_PRIO_LATENCY=1
run X=0
