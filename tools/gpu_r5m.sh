#!/bin/bash
# round-5: the O=15 sequence GPU tests, then the default bench line
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sequence.py -x -q --timeout 300 --timeout-method thread -k "15" > gpurun_out/r5m_tests.log 2>&1 || { tail -20 gpurun_out/r5m_tests.log; exit 1; }
tail -1 gpurun_out/r5m_tests.log
timeout -k 10 600 python -u bench.py > gpurun_out/r5m_bench.json 2> gpurun_out/r5m_bench.err || { tail -5 gpurun_out/r5m_bench.err; exit 1; }
tail -1 gpurun_out/r5m_bench.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d.get('sequence') or {}
print('value', d['value'], 'ms', d['ms_per_step'], 'ok', d['chains_ok'], 'boot', d.get('bootstrap_s'), 'seq00', d.get('seq00_frames_per_s'))
print('vs_ref', {k: (d.get('headline_vs_reference') or {}).get(k) for k in ('compared','identical')})
print('seq', {k: s.get(k) for k in ('frames_per_s','wall_s_runs','shards','bootstrap_s','steps','ms_per_step','vs_reference','stitched_ate_rel_vs_gt','stitch_ms')})
for w, r in (s.get('rank_slices') or {}).items(): print('slice', w, {k: r.get(k) for k in ('shards_total','per_rank_wall_s','wall_s_runs','predicted_frames_per_s','predicted_frames_per_s_incl_stitch','shards_identical')})
print('single', d.get('single_chain')); print('roof', d.get('roofline')); print('cpu', d.get('cpu_baseline'))
print('c3', d.get('c3_sift_match')); print('c5', d.get('c5_hd1080')); print('matcher', (d.get('roofline_matcher') or {}).get('frac'))"
