#!/bin/bash
# A/B of the in-tree library against _build/libvo_base.so on the latency legs: single chain
# (eager / graph), the one-GPU sequence job and the rank slices, plus the headline; alternating.
# usage: bash tools/gpu_seqab.sh <tag> <reps>
tag=$1; reps=$2
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
BASE=$PWD/monocular_visual_odometry_va4mr_amd/_build/libvo_base.so
out=gpurun_out/${tag}_seqab.jsonl; : > $out
run() { local name=$1; shift; env "$@" timeout -k 10 400 python -u bench.py --no-match --no-cpu --steps 20 --warmup 5 > gpurun_out/sab.json 2> gpurun_out/sab.err || { tail -5 gpurun_out/sab.err; return 1; }
  tail -1 gpurun_out/sab.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d.get('sequence') or {}; sc=d.get('single_chain') or {}
rs={k: v.get('predicted_frames_per_s') for k, v in (s.get('rank_slices') or {}).items()}
print(json.dumps({'lib': '$name', 'value': d['value'], 'ms': d['ms_per_step'], 'ok': d['chains_ok'], 'vs_ref': (d.get('headline_vs_reference') or {}).get('identical'),
  'pnp_ms': (d.get('stages_ms') or {}).get('pnp'), 'single': sc.get('frames_per_s'), 'single_graph': sc.get('graph_frames_per_s'), 'graph_identical': sc.get('graph_identical'),
  'seq00': s.get('frames_per_s'), 'seq_identical': (s.get('vs_reference') or {}).get('shards_identical'), 'slices': rs, 'boot': d.get('bootstrap_s')}))" | tee -a $out; }
for i in $(seq $reps); do run new VO_X=1 && run base VO_HIP_LIB=$BASE || exit 1; done
