#!/bin/bash
# round-4 probe: sequence job sweep (shards x stream groups) and the LK per-level phase profile
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/seq_sweep.py 32 64 128 --groups 1,2 > gpurun_out/seqsweep_r4b.jsonl 2> gpurun_out/seqsweep_r4b.err || { tail -5 gpurun_out/seqsweep_r4b.err; exit 1; }
cut -c1-700 gpurun_out/seqsweep_r4b.jsonl
timeout -k 10 200 python -u tools/lk_prof.py 30 > gpurun_out/lkprof_r4.txt 2>&1 || { tail -5 gpurun_out/lkprof_r4.txt; exit 1; }
cat gpurun_out/lkprof_r4.txt
