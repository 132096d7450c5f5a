#!/bin/bash
# next-step pyramid prefetch: sequence / headline / step tests, then A/B against VO_PREFETCH=0
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_sequence.py tests/test_gpu_headline.py tests/test_gpu_step_paths.py tests/test_gpu_shards.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6r_tests.log 2>&1 || { tail -30 gpurun_out/r6r_tests.log; exit 1; }
tail -1 gpurun_out/r6r_tests.log
out=gpurun_out/r6r_ab.jsonl; : > $out
run() { local name=$1; shift; env "$@" timeout -k 10 400 python -u bench.py --no-match --no-cpu --no-single --steps 30 --warmup 5 > gpurun_out/sab.json 2> gpurun_out/sab.err || { tail -5 gpurun_out/sab.err; return 1; }
  tail -1 gpurun_out/sab.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d.get('sequence') or {}
rs={k: v.get('predicted_frames_per_s') for k, v in (s.get('rank_slices') or {}).items()}
ri={k: v.get('shards_identical') for k, v in (s.get('rank_slices') or {}).items()}
print(json.dumps({'cfg': '$name', 'value': d['value'], 'ms': d['ms_per_step'], 'ok': d['chains_ok'], 'vs_ref': (d.get('headline_vs_reference') or {}).get('identical'),
  'seq00': s.get('frames_per_s'), 'seq_identical': (s.get('vs_reference') or {}).get('shards_identical'), 'slices': rs, 'slices_identical': ri, 'stages': d.get('stages_ms')}))" | tee -a $out; }
for i in 1 2; do run prefetch VO_X=1 && run noprefetch VO_PREFETCH=0 || exit 1; done
