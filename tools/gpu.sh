#!/bin/bash
# One parametrised GPU runner (replaces the per-round gpu_r*.sh scripts).  Run through gpurun:
#   bash tools/gpu.sh tests  <tag> [pytest args]      -m gpu tests (default: the whole suite)
#   bash tools/gpu.sh bench  <tag> [bench args]       one bench line -> gpurun_out/<tag>.json
#   bash tools/gpu.sh ab     <tag> <reps> <A env> <B env> [bench args]
#                                                     headline A/B alternating two env settings,
#                                                     e.g. VO_SEL_SPLIT=1 VO_SEL_SPLIT=0 (AB_ARGS replaces
#                                                     the default headline-only flags)
#   bash tools/gpu.sh abargs <tag> <reps> "<flags A>" "<flags B>"   the same over two bench flag sets
#   bash tools/gpu.sh timeline <tag> [bench args]     per-queue kernel timeline of the headline
#   bash tools/gpu.sh trace  <tag> [bench args]       kernel-trace stats of a bench run (by grid)
#   bash tools/gpu.sh pmc    <tag>                    FETCH/WRITE + k_lk_w SQ counter passes
#   bash tools/gpu.sh smoke  <tag>                    __graft_entry__.smoke()
# Several commands can be chained in one call with '&&'; each step has its own time limit.
set -o pipefail
what=$1; tag=$2; shift 2
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
O=gpurun_out
HL="--no-cpu --no-single --no-match --no-sequence"
summ() {   # one-line summary of a bench JSON line
python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d.get('sequence') or {}; r=d.get('roofline') or {}
print(json.dumps({'tag': sys.argv[2], 'value': d['value'], 'ms': d['ms_per_step'], 'ok': d.get('chains_ok'), 'lk_ms': r.get('mean_ms'),
  'stages': d.get('stages_ms'), 'vs_ref': [(d.get('headline_vs_reference') or {}).get(k) for k in ('compared', 'identical')],
  'boot': d.get('bootstrap_s'), 'seq00': d.get('seq00_frames_per_s'),
  'slices': {w: x.get('predicted_frames_per_s') for w, x in (s.get('rank_slices') or {}).items() if isinstance(x, dict)},
  'single': [(d.get('single_chain') or {}).get(k) for k in ('frames_per_s', 'graph_frames_per_s')],
  'c5': (d.get('c5_hd1080') or {}).get('frames_per_s'), 'c3': (d.get('c3_sift_match') or {}).get('pairs_per_s'),
  'matcher': (d.get('roofline_matcher') or {}).get('frac')}))" "$@"
}
case $what in
tests)
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > $O/${tag}_tests.log 2>&1
  rc=$?; tail -3 $O/${tag}_tests.log; exit $rc ;;
smoke)
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/${tag}_smoke.log 2>&1
  rc=$?; tail -2 $O/${tag}_smoke.log; exit $rc ;;
bench)
  timeout -k 10 900 python -u bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }
  summ $O/$tag.json $tag ;;
ab)
  reps=$1; A=$2; B=$3; shift 3
  out=$O/${tag}_ab.jsonl; : > $out
  for i in $(seq $reps); do
    for E in "$A" "$B"; do
      env $E timeout -k 10 300 python -u bench.py ${AB_ARGS:-$HL} --steps 20 --warmup 5 "$@" > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
      summ $O/ab.json "$E" | tee -a $out
    done
  done ;;
abn)       # headline runs cycling over any number of env settings: abn <tag> <reps> "<env 1>" "<env 2>" ...
  reps=$1; shift
  out=$O/${tag}_ab.jsonl; : > $out
  for i in $(seq $reps); do
    for E in "$@"; do
      env $E timeout -k 10 300 python -u bench.py ${AB_ARGS:-$HL} --steps 20 --warmup 5 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
      summ $O/ab.json "$E" | tee -a $out
    done
  done ;;
abargs)    # headline A/B alternating two bench flag sets: abargs <tag> <reps> "<flags A>" "<flags B>"
  reps=$1; A=$2; B=$3; shift 3
  out=$O/${tag}_ab.jsonl; : > $out
  for i in $(seq $reps); do
    for F in "$A" "$B"; do
      timeout -k 10 300 python -u bench.py ${AB_ARGS:-$HL} --steps 20 --warmup 5 $F > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
      summ $O/ab.json "$F" | tee -a $out
    done
  done ;;
timeline)
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl_$tag -o run -- python bench.py $HL --steps 6 --warmup 3 "$@" > $O/tl_$tag.log 2>&1 || exit $?
  python3 tools/timeline.py $O/tl_$tag > $O/tl_$tag.txt
  rm -f $O/tl_$tag/*kernel_trace.csv.bak
  head -60 $O/tl_$tag.txt ;;
slab)      # sequence rank slices cycling over env settings: slab <tag> <reps> <W:B:O> "<env 1>" "<env 2>" ...
  reps=$1; spec=$2; shift 2
  out=$O/${tag}_slab.jsonl; : > $out
  for i in $(seq $reps); do
    for E in "$@"; do
      env $E timeout -k 10 300 python -u tools/slice_sweep.py $spec --reps 3 2> $O/slab.err | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); d['tag']=sys.argv[1]; print(json.dumps(d))" "$E" | tee -a $out || { tail -20 $O/slab.err; exit 1; }
    done
  done ;;
slicetl)   # kernel timeline + by-grid stats of one sequence rank slice: slicetl <tag> <W:B:O>
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/stl_$tag -o run -- python tools/slice_sweep.py ${1:-8:24:15} --reps 1 > $O/stl_$tag.log 2>&1 || exit $?
  python3 tools/timeline.py $O/stl_$tag 1600 > $O/stl_$tag.txt
  python3 tools/trace_by_grid.py $O/stl_$tag $O/stl_${tag}_by_grid.csv
  rm -f $O/stl_$tag/*kernel_trace.csv
  tail -2 $O/stl_$tag.log; head -25 $O/stl_${tag}_by_grid.csv ;;
trace)
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$tag -o run -- python bench.py "$@" > $O/prof_$tag.json 2> $O/prof_$tag.err || exit $?
  python3 tools/trace_by_grid.py $O/prof_$tag $O/prof_${tag}_by_grid.csv
  rm -f $O/prof_$tag/*kernel_trace.csv
  head -30 $O/prof_${tag}_by_grid.csv ;;
pmc)
  K="--kernel-include-regex ::k_"; R="--output-format csv"; KL="--kernel-include-regex k_lk_w"
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE $K $R -d $O/pmc_fetch_$tag -o run -- python bench.py $HL > $O/pmc_fetch_$tag.json 2>&1 || exit $?
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE $K $R -d $O/pmc_write_$tag -o run -- python bench.py $HL > $O/pmc_write_$tag.json 2>&1 || exit $?
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY $KL $R -d $O/sq1_$tag -o run -- python bench.py $HL > $O/sq1_$tag.json 2>&1 || exit $?
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE $KL $R -d $O/sq2_$tag -o run -- python bench.py $HL > $O/sq2_$tag.json 2>&1 || exit $?
  du -sh $O/*_$tag* | tail -8 ;;
*) echo "unknown command $what"; exit 2 ;;
esac
