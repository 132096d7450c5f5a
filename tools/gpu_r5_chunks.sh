#!/bin/bash
# round-5 A/B: the headline with the LK grid split into n launches (VO_LK_CHUNKS), alternating
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
out=gpurun_out/r5_chunks.jsonl
: > $out
for rep in 1 2; do
  for n in ${CHUNKS:-1 2 4 8}; do
    VO_LK_CHUNKS=$n timeout -k 10 200 python -u bench.py --no-sequence --no-single --no-match --no-cpu --steps 20 --warmup 5 > gpurun_out/ch.json 2> gpurun_out/ch.err || { tail -5 gpurun_out/ch.err; exit 1; }
    tail -1 gpurun_out/ch.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
r={'chunks': $n, 'value': d['value'], 'ms': d['ms_per_step'], 'ok': d['chains_ok'], 'stages': d['stages_ms'], 'vs_ref': {k: (d.get('headline_vs_reference') or {}).get(k) for k in ('compared','identical')}}
print(json.dumps(r))" | tee -a $out
  done
done
