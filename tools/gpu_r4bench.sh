#!/bin/bash
# round-4 default bench line + kernel-trace summary of the same command (profiles/r4*)
tag=${1:-r4a}
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || { tail -5 gpurun_out/bench_$tag.err; exit 1; }
tail -1 gpurun_out/bench_$tag.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('value', d['value'], 'ms', d['ms_per_step'], 'ok', d['chains_ok'], 'boot', d['bootstrap_s'], 'seq00', d.get('seq00_frames_per_s'))
print('single', d.get('single_chain')); print('seq', {k: d['sequence'].get(k) for k in ('frames_per_s','wall_s','bootstrap_s','ms_per_step','shards','groups','shards_ok','vs_reference')})
print('roof', d['roofline']); print('cpu', d.get('cpu_baseline'))
for k in ('c3_sift_match','c5_sift_match','c5_hd1080'): print(k, {kk: vv for kk, vv in (d.get(k) or {}).items() if kk in ('frames_per_s','pairs_per_s','sift_ms_per_image','bf_ms_per_pair','ms_per_step','error')})
print('matcher', d.get('roofline_matcher', {}).get('frac'))"
