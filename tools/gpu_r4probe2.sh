#!/bin/bash
# round-4 probe 2: LK per-iteration cost; PnP micro phases; sequence job (workspace reserved
# before the clock) over stream groups / priority / one-stream engines; kernel trace of the
# 64-chain job
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 60 ./tools/micro/pnp_micro 10 > gpurun_out/pnp_micro_r4.txt 2>&1; tail -8 gpurun_out/pnp_micro_r4.txt
timeout -k 10 300 python -u tools/lk_iter_cost.py 1 16 384 > gpurun_out/lkiter_r4.jsonl 2> gpurun_out/lkiter_r4.err || { tail -5 gpurun_out/lkiter_r4.err; exit 1; }
cat gpurun_out/lkiter_r4.jsonl
for cfg in "1 0" "0 0" "1 1"; do
  set -- $cfg
  VO_SEQ_PRIO=$1 VO_ONE_STREAM=$2 timeout -k 10 300 python -u tools/seq_sweep.py 64 --groups 1,2,3,4 > gpurun_out/seqsweep_r4c_$1$2.jsonl 2> gpurun_out/seqsweep_r4c.err || { tail -5 gpurun_out/seqsweep_r4c.err; exit 1; }
  echo "prio $1 one_stream $2"
  python3 -c "
import json,sys
for l in open('gpurun_out/seqsweep_r4c_$1$2.jsonl'):
    d=json.loads(l); print(d['chains_per_gpu'], d['groups'], d['sequence_frames_per_s'], d['wall_s'], d['bootstrap_s'], d['ms_per_step'], d['shards_ok'], (d.get('vs_reference') or {}).get('shards_identical'))"
done
rm -rf gpurun_out/seqprof
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d gpurun_out/seqprof -o seq -- python3 tools/seq_sweep.py 64 --groups 2 > gpurun_out/seqprof.log 2>&1 || { tail -5 gpurun_out/seqprof.log; exit 1; }
python3 tools/trace_by_grid.py gpurun_out/seqprof gpurun_out/seqprof_by_grid.csv && head -30 gpurun_out/seqprof_by_grid.csv
python3 tools/timeline.py gpurun_out/seqprof 160 > gpurun_out/seqprof_timeline.txt
