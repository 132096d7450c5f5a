#!/bin/bash
# whole-sequence job vs shards per GPU (tools/seq_sweep.py).  usage: gpu_seqsweep.sh <tag> [B ...]
tag=${1:-r4}; shift
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/seq_sweep.py "$@" > gpurun_out/seqsweep_$tag.jsonl 2> gpurun_out/seqsweep_$tag.err
rc=$?
cat gpurun_out/seqsweep_$tag.jsonl | cut -c1-600
tail -3 gpurun_out/seqsweep_$tag.err
exit $rc
