#!/bin/bash
# round-5: wave-shaped feature adding (k_add_w) -- parity tests, headline A/B vs k_add_finish
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_step_paths.py tests/test_gpu_headline.py tests/test_gpu_configs.py > gpurun_out/r5g_tests.log 2>&1 || { tail -30 gpurun_out/r5g_tests.log; exit 1; }
tail -2 gpurun_out/r5g_tests.log
out=gpurun_out/r5g_ab.jsonl; : > $out
hl() { local v=$1; VO_ADD_WAVE=$v timeout -k 10 200 python -u bench.py --no-sequence --no-single --no-match --no-cpu --steps 20 --warmup 5 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; return 1; }
  tail -1 gpurun_out/ab.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print(json.dumps({'add_wave': $v, 'value': d['value'], 'ms': d['ms_per_step'], 'ok': d['chains_ok'], 'vs_ref': [(d.get('headline_vs_reference') or {}).get(k) for k in ('compared','identical')]}))" | tee -a $out; }
hl 1 && hl 0 && hl 1 && hl 0 || exit 1
