#!/bin/bash
# pyramid build alone: events + kernel-trace stats by launch shape.  usage: bash tools/gpu_pyr.sh <tag>
tag=${1:-p}
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 240 python tools/pyr_bench.py 16 384 768 > gpurun_out/pyr_$tag.jsonl 2> gpurun_out/pyr_$tag.err || { tail -5 gpurun_out/pyr_$tag.err; exit 1; }
cat gpurun_out/pyr_$tag.jsonl
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pk_$tag -o run -- python tools/pyr_bench.py 384 > gpurun_out/pk_$tag.log 2>&1 || { tail -5 gpurun_out/pk_$tag.log; exit 1; }
python tools/trace_by_grid.py gpurun_out/pk_$tag gpurun_out/pk_$tag/by_grid.csv && rm -f gpurun_out/pk_$tag/*kernel_trace.csv
head -12 gpurun_out/pk_$tag/by_grid.csv
