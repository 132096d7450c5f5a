#!/bin/bash
# single chain (drop-in class mode): latency, kernel trace of the graph-replayed loop, and the
# PnP micro-benchmark breakdown.  usage: gpu_single.sh <tag>
set -e
tag=${1:-a}
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 200 python -u tools/single_prof.py 200 > gpurun_out/single_${tag}.log 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/single_${tag}_t -o run -- python3 tools/single_prof.py 200 >> gpurun_out/single_${tag}.log 2>&1
if [ -x tools/micro/pnp_micro ]; then timeout -k 10 60 tools/micro/pnp_micro >> gpurun_out/single_${tag}.log 2>&1; fi
