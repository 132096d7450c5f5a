#!/bin/bash
# Headline A/B of the in-tree library against _build/libvo_base.so (tools/build_ab.sh), alternating,
# after the given GPU tests.  usage: bash tools/gpu_ab.sh <tag> <reps> [pytest args...]
tag=$1; reps=$2; shift 2
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
BASE=$PWD/monocular_visual_odometry_va4mr_amd/_build/libvo_base.so
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu "$@" > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
  tail -1 gpurun_out/${tag}_tests.log
fi
out=gpurun_out/${tag}_ab.jsonl; : > $out
hl() { local name=$1; shift; env "$@" timeout -k 10 200 python -u bench.py --no-sequence --no-single --no-match --no-cpu --steps 20 --warmup 5 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; return 1; }
  tail -1 gpurun_out/ab.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}
print(json.dumps({'lib': '$name', 'value': d['value'], 'ms': d['ms_per_step'], 'ok': d['chains_ok'], 'lk_ms': r.get('mean_ms'), 'vs_ref': [(d.get('headline_vs_reference') or {}).get(k) for k in ('compared','identical')]}))" | tee -a $out; }
for i in $(seq $reps); do hl new VO_X=1 && hl base VO_HIP_LIB=$BASE || exit 1; done
