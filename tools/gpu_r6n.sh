#!/bin/bash
# headline with the select block at 512 (default) / 256 / 1024 threads, after k_add_finish_lean
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
out=gpurun_out/r6n_sel.jsonl; : > $out
hl() { local name=$1; shift; env "$@" timeout -k 10 200 python -u bench.py --no-sequence --no-single --no-match --no-cpu --steps 20 --warmup 5 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; return 1; }
  tail -1 gpurun_out/ab.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print(json.dumps({'cfg': '$name', 'value': d['value'], 'ms': d['ms_per_step'], 'ok': d['chains_ok'], 'stages': d.get('stages_ms')}))" | tee -a $out; }
for i in 1 2; do hl sel512 VO_X=1 && hl sel256 VO_SEL_THREADS=256 && hl sel1024 VO_SEL_THREADS=1024 || exit 1; done
