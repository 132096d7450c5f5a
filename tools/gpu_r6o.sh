#!/bin/bash
# headline with k_pnp_tri built for 4 waves per SIMD (128 VGPRs, spilled) vs the 2-wave build
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
W4=$PWD/monocular_visual_odometry_va4mr_amd/_build/libvo_wpe4.so
VO_HIP_LIB=$W4 timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6o_tests.log 2>&1 || { tail -20 gpurun_out/r6o_tests.log; exit 1; }
tail -1 gpurun_out/r6o_tests.log
out=gpurun_out/r6o_ab.jsonl; : > $out
hl() { local name=$1; shift; env "$@" timeout -k 10 200 python -u bench.py --no-sequence --no-single --no-match --no-cpu --steps 30 --warmup 5 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; return 1; }
  tail -1 gpurun_out/ab.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print(json.dumps({'cfg': '$name', 'value': d['value'], 'ms': d['ms_per_step'], 'ok': d['chains_ok'], 'vs_ref': (d.get('headline_vs_reference') or {}).get('identical'), 'stages': d.get('stages_ms')}))" | tee -a $out; }
for i in 1 2; do hl wpe4 VO_HIP_LIB=$W4 && hl wpe2 VO_X=1 || exit 1; done
