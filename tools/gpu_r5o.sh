#!/bin/bash
# round-5: stream groups at the headline (768 chains) after the row-streaming pyramid
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
out=gpurun_out/r5o_groups.jsonl; : > $out
hl() { local g=$1; timeout -k 10 200 python -u bench.py --no-sequence --no-single --no-match --no-cpu --steps 20 --warmup 5 --groups $g > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; return 1; }
  tail -1 gpurun_out/ab.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print(json.dumps({'groups': $g, 'value': d['value'], 'ms': d['ms_per_step'], 'ok': d['chains_ok']}))" | tee -a $out; }
hl 2 && hl 3 && hl 4 && hl 1 && hl 2 && hl 3 && hl 4 || exit 1
