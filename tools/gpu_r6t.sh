#!/bin/bash
# headline / sequence with the next-step pyramid on a stream of its own (VO_PREFETCH=2) vs default
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
VO_PREFETCH=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_sequence.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6t_tests.log 2>&1 || { tail -30 gpurun_out/r6t_tests.log; exit 1; }
tail -1 gpurun_out/r6t_tests.log
out=gpurun_out/r6t_ab.jsonl; : > $out
run() { local name=$1; shift; env "$@" timeout -k 10 400 python -u bench.py --no-match --no-cpu --no-single --no-rank-slices --steps 30 --warmup 5 > gpurun_out/sab.json 2> gpurun_out/sab.err || { tail -5 gpurun_out/sab.err; return 1; }
  tail -1 gpurun_out/sab.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d.get('sequence') or {}
print(json.dumps({'cfg': '$name', 'value': d['value'], 'ms': d['ms_per_step'], 'ok': d['chains_ok'], 'vs_ref': (d.get('headline_vs_reference') or {}).get('identical'),
  'seq00': s.get('frames_per_s'), 'seq_identical': (s.get('vs_reference') or {}).get('shards_identical'), 'stages': d.get('stages_ms')}))" | tee -a $out; }
for i in 1 2; do run own VO_PREFETCH=2 && run default VO_X=1 || exit 1; done
