#!/bin/bash
# matcher launch fusion: matcher / SIFT GPU tests, then the C3 / C5 legs of the bench
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bootstrap.py tests/test_gpu_configs.py -m gpu > gpurun_out/r4match_tests.log 2>&1 || { tail -20 gpurun_out/r4match_tests.log; exit 1; }
tail -1 gpurun_out/r4match_tests.log
timeout -k 10 400 python -u bench.py --no-cpu --no-single --no-sequence --steps 10 --warmup 3 > gpurun_out/r4match.json 2> gpurun_out/r4match.err || { tail -5 gpurun_out/r4match.err; exit 1; }
tail -1 gpurun_out/r4match.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('value', d['value'], 'boot', d['bootstrap_s'])
for k in ('c3_sift_match','c5_sift_match'): print(k, {kk: vv for kk, vv in (d.get(k) or {}).items() if kk in ('pairs_per_s','sift_ms_per_image','bf_ms_per_pair','error')}, (d.get(k) or {}).get('bf_roofline',{}).get('frac'))
print('matcher', d.get('roofline_matcher', {}).get('frac'), 'c5', (d.get('c5_hd1080') or {}).get('frames_per_s'))"
