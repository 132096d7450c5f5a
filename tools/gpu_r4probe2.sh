#!/bin/bash
# round-4 probe 2: LK per-iteration cost; sequence job with the workspace reserved before the
# clock, with and without the high-priority first group; kernel trace of the 64-chain job
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/lk_iter_cost.py 1 16 384 > gpurun_out/lkiter_r4.jsonl 2> gpurun_out/lkiter_r4.err || { tail -5 gpurun_out/lkiter_r4.err; exit 1; }
cat gpurun_out/lkiter_r4.jsonl
for p in 1 0; do
  VO_SEQ_PRIO=$p timeout -k 10 300 python -u tools/seq_sweep.py 32 64 --groups 1,2 > gpurun_out/seqsweep_r4c_p$p.jsonl 2> gpurun_out/seqsweep_r4c.err || { tail -5 gpurun_out/seqsweep_r4c.err; exit 1; }
  echo "prio $p"; cut -c1-160,400-720 gpurun_out/seqsweep_r4c_p$p.jsonl
done
# kernel trace of the 64-chain, 2-group sequence job (one sweep point)
rm -rf gpurun_out/seqprof
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d gpurun_out/seqprof -o seq -- python3 tools/seq_sweep.py 64 --groups 2 > gpurun_out/seqprof.log 2>&1 || { tail -5 gpurun_out/seqprof.log; exit 1; }
python3 tools/trace_by_grid.py gpurun_out/seqprof gpurun_out/seqprof_by_grid.csv && head -30 gpurun_out/seqprof_by_grid.csv
python3 tools/timeline.py gpurun_out/seqprof 120 > gpurun_out/seqprof_timeline.txt
