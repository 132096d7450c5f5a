#!/bin/bash
# round-5: row-streaming pyramid (k_pyr_rows) -- parity tests, pyramid alone, headline A/B vs the tile kernels
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "pyramid or lk or step" > gpurun_out/r5f_tests.log 2>&1 || { tail -30 gpurun_out/r5f_tests.log; exit 1; }
tail -2 gpurun_out/r5f_tests.log
for v in 1 0; do VO_PYR_ROWS=$v timeout -k 10 200 python tools/pyr_bench.py 16 384 768 | sed "s/^/rows=$v /" || exit 1; done
out=gpurun_out/r5f_ab.jsonl; : > $out
hl() { local v=$1; VO_PYR_ROWS=$v timeout -k 10 200 python -u bench.py --no-sequence --no-single --no-match --no-cpu --steps 20 --warmup 5 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; return 1; }
  tail -1 gpurun_out/ab.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print(json.dumps({'rows': $v, 'value': d['value'], 'ms': d['ms_per_step'], 'ok': d['chains_ok'], 'vs_ref': [(d.get('headline_vs_reference') or {}).get(k) for k in ('compared','identical')]}))" | tee -a $out; }
hl 1 && hl 0 && hl 1 && hl 0 || exit 1
