#!/bin/bash
# round-5: SIFT descriptor walk with LDS float atomics -- SIFT parity tests, sift_bench + headline bootstrap A/B
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
BASE=$PWD/monocular_visual_odometry_va4mr_amd/_build/libvo_base.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bootstrap.py tests/test_gpu_configs.py -k "sift or bootstrap or c5" > gpurun_out/${TAG:-r5p}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG:-r5p}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG:-r5p}_tests.log
out=gpurun_out/${TAG:-r5p}_ab.jsonl; : > $out
sb() { local tag=$1; shift; env "$@" timeout -k 10 200 python -u tools/sift_bench.py 3 kitti 2> gpurun_out/sb.err | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); d['tag']='$tag'; print(json.dumps(d))" | tee -a $out; }
hl() { local tag=$1; shift; env "$@" timeout -k 10 200 python -u bench.py --no-sequence --no-single --no-match --no-cpu --steps 10 --warmup 3 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; return 1; }
  tail -1 gpurun_out/ab.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print(json.dumps({'tag': '$tag', 'bootstrap_s': d['bootstrap_s'], 'value': d['value'], 'vs_ref': [(d.get('headline_vs_reference') or {}).get(k) for k in ('compared','identical')], 'ok': d['chains_ok']}))" | tee -a $out; }
sb new VO_X=1 && sb base VO_HIP_LIB=$BASE && sb new VO_X=1 && sb base VO_HIP_LIB=$BASE || exit 1
hl new VO_X=1 && hl base VO_HIP_LIB=$BASE && hl new VO_X=1 && hl base VO_HIP_LIB=$BASE || exit 1
