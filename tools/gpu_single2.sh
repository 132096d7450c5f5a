#!/bin/bash
# single chain (drop-in class mode): latency, then kernel traces of the fused (default) and the
# split PnP / triangulation launches, with the per-queue timeline of the last graph steps.
# usage: gpu_single2.sh <tag>
set -e
tag=${1:-a}
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
L=gpurun_out/single2_${tag}.log
timeout -k 10 200 python -u tools/single_prof.py 200 > $L 2>&1
VO_PNP_TRI_SPLIT=1 timeout -k 10 200 python -u tools/single_prof.py 200 >> $L 2>&1
for v in 0 1; do
  export VO_PNP_TRI_SPLIT=$v
  timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/single2_${tag}_$v -o run -- python3 tools/single_prof.py 120 >> $L 2>&1
  python3 tools/trace_by_grid.py gpurun_out/single2_${tag}_$v gpurun_out/single2_${tag}_${v}_by_grid.csv
  python3 tools/timeline.py gpurun_out/single2_${tag}_$v 40 > gpurun_out/single2_${tag}_${v}_timeline.txt
  find gpurun_out/single2_${tag}_$v -name "*kernel_trace.csv" -delete
done
