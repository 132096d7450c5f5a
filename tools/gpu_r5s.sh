#!/bin/bash
# round-5: LK launch knobs at the headline (XCD-grouped block map, blocks per chain)
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
out=gpurun_out/r5s_lk_knobs.jsonl; : > $out
hl() { local tag=$1; shift; env "$@" timeout -k 10 200 python -u bench.py --no-sequence --no-single --no-match --no-cpu --steps 20 --warmup 5 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; return 1; }
  tail -1 gpurun_out/ab.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print(json.dumps({'tag': '$tag', 'value': d['value'], 'ms': d['ms_per_step'], 'ok': d['chains_ok']}))" | tee -a $out; }
for i in 1 2; do
hl base VO_X=1 && hl xcd VO_LK_XCD=1 && hl nb1024 VO_LK_NB=1024 && hl nb3072 VO_LK_NB=3072 || exit 1
done
