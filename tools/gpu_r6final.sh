#!/bin/bash
# round-5 final: smoke, the default bench line twice
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6final_smoke.log 2>&1 || { tail -20 gpurun_out/r6final_smoke.log; exit 1; }
tail -1 gpurun_out/r6final_smoke.log
for i in 1 2; do
timeout -k 10 600 python -u bench.py > gpurun_out/r6final_bench_$i.json 2> gpurun_out/r6final_bench_$i.err || { tail -5 gpurun_out/r6final_bench_$i.err; exit 1; }
tail -1 gpurun_out/r6final_bench_$i.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d.get('sequence') or {}
print('value', d['value'], 'ms', d['ms_per_step'], 'ok', d['chains_ok'], 'boot', d.get('bootstrap_s'), 'seq00', d.get('seq00_frames_per_s'), 'vs_ref', (d.get('headline_vs_reference') or {}).get('identical'))
print('slices', {w: r.get('predicted_frames_per_s') for w, r in (s.get('rank_slices') or {}).items()}, 'single', (d.get('single_chain') or {}).get('frames_per_s'), (d.get('single_chain') or {}).get('graph_frames_per_s'))
print('c5', (d.get('c5_hd1080') or {}).get('frames_per_s'), 'c3', (d.get('c3_sift_match') or {}).get('pairs_per_s'), 'matcher', (d.get('roofline_matcher') or {}).get('frac'), 'roof', d['roofline']['frac'], 'cpu', d['cpu_baseline']['value'])"
done
