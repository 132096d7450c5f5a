#!/bin/bash
# round-5 A/B: k_lk_w I-window quads (default) vs the round-4 byte rows (libvo_lkbytes.so) at the
# headline and at C5; LK chunked launches; kernel trace of the default bench (profiles/r5a_*)
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
BYTES=$PWD/monocular_visual_odometry_va4mr_amd/_build/libvo_lkbytes.so
hl() {  # tag, then env assignments
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-sequence --no-single --no-match --no-cpu --steps 20 --warmup 5 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; return 1; }
  tail -1 gpurun_out/ab.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print(json.dumps({'tag': '$tag', 'value': d['value'], 'ms': d['ms_per_step'], 'ok': d['chains_ok'], 'track_ms': d['stages_ms']['track'], 'stages': d['stages_ms'], 'vs_ref': [(d.get('headline_vs_reference') or {}).get(k) for k in ('compared','identical')]}))" | tee -a gpurun_out/r5b_ab.jsonl
}
c5() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u tools/c5_only.py 256 2 > gpurun_out/c5ab.json 2> gpurun_out/c5ab.err || { tail -5 gpurun_out/c5ab.err; return 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c5ab.json').read().splitlines()[-1]); d['tag']='$tag'; print(json.dumps(d))" | tee -a gpurun_out/r5b_ab.jsonl
}
: > gpurun_out/r5b_ab.jsonl
hl quads VO_X=1 && hl bytes VO_HIP_LIB=$BYTES && hl quads VO_X=1 && hl bytes VO_HIP_LIB=$BYTES || exit 1
c5 c5_quads VO_X=1 && c5 c5_bytes VO_HIP_LIB=$BYTES && c5 c5_quads VO_X=1 && c5 c5_bytes VO_HIP_LIB=$BYTES || exit 1
hl chunks2 VO_LK_CHUNKS=2 && hl chunks4 VO_LK_CHUNKS=4 && hl chunks1 VO_LK_CHUNKS=1 || exit 1
rm -rf gpurun_out/prof5
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof5 -o r5 -- python3 bench.py > gpurun_out/r5a_prof_bench.json 2> gpurun_out/r5a_prof_bench.err || { tail -5 gpurun_out/r5a_prof_bench.err; exit 1; }
python3 tools/trace_by_grid.py gpurun_out/prof5 gpurun_out/r5a_by_grid.csv && head -24 gpurun_out/r5a_by_grid.csv
find gpurun_out/prof5 -name "*kernel_stats.csv" -exec cp {} gpurun_out/r5a_kernel_stats.csv \;
rm -rf gpurun_out/prof5
