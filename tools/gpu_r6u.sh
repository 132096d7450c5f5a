#!/bin/bash
# final tree (round 5): full GPU suite, smoke, one default bench
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6u_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r6u_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r6u_gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6u_smoke.log 2>&1 || { tail -20 gpurun_out/r6u_smoke.log; exit 1; }
tail -1 gpurun_out/r6u_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r6u_bench.json 2> gpurun_out/r6u_bench.err || { tail -5 gpurun_out/r6u_bench.err; exit 1; }
tail -1 gpurun_out/r6u_bench.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['sequence']; sc=d['single_chain']
print('value', d['value'], 'ms', d['ms_per_step'], 'ok', d['chains_ok'], 'vs_ref', d['headline_vs_reference']['identical'], 'seq00', d['seq00_frames_per_s'],
 'slices', {k: v['predicted_frames_per_s'] for k, v in s['rank_slices'].items()}, 'single', sc['frames_per_s'], sc['graph_frames_per_s'], 'c5', d['c5_hd1080']['frames_per_s'], 'boot', d['bootstrap_s'])"
