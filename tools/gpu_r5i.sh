#!/bin/bash
# round-5: pyramid lookahead (Engine.enable_lookahead) -- step-path + headline tests, headline A/B
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_step_paths.py tests/test_gpu_headline.py > gpurun_out/r5i_tests.log 2>&1 || { tail -30 gpurun_out/r5i_tests.log; exit 1; }
tail -1 gpurun_out/r5i_tests.log
out=gpurun_out/r5i_ab.jsonl; : > $out
hl() { local v=$1; VO_LOOKAHEAD=$v timeout -k 10 200 python -u bench.py --no-sequence --no-single --no-match --no-cpu --steps 20 --warmup 5 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; return 1; }
  tail -1 gpurun_out/ab.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print(json.dumps({'lookahead': $v, 'value': d['value'], 'ms': d['ms_per_step'], 'ok': d['chains_ok'], 'vs_ref': [(d.get('headline_vs_reference') or {}).get(k) for k in ('compared','identical')]}))" | tee -a $out; }
hl 1 && hl 0 && hl 1 && hl 0 || exit 1
