#!/bin/bash
# sequence job (64 shards, 2 groups): a device sync after the bootstraps (time_boot) or none
# (each group steps as soon as its own bootstrap is done), alternating
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
: > gpurun_out/bootsync.jsonl
for rep in 1 2 3; do
  for f in "" --no-boot-sync; do
    timeout -k 10 300 python -u tools/seq_sweep.py --groups 2 --reps 2 $f 64 > gpurun_out/bs_one.jsonl 2> gpurun_out/bs.err || { tail -5 gpurun_out/bs.err; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/bs_one.jsonl'):
    d=json.loads(l); d['flag']='$f'; print(json.dumps(d))
    print('flag=$f', {k: d.get(k) for k in ('sequence_frames_per_s','wall_s','bootstrap_s','ms_per_step','shards_ok')}, d.get('vs_reference',{}).get('shards_identical'))" | tee -a gpurun_out/bootsync.jsonl | grep "^flag="
  done
done
