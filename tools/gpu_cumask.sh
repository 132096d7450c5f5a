#!/bin/bash
# Headline bench (768 chains) with the LK launches on CU-masked streams: sweep the number of
# CUs left free for the latency-bound stages and the stream-group count.
# usage: bash tools/gpu_cumask.sh <tag> "<reserve list>" "<groups list>"
tag=${1:-cm}
res=${2:-"0 16 32 64"}
grp=${3:-"2"}
mkdir -p gpurun_out
out=gpurun_out/cumask_$tag.txt
: > $out
for g in $grp; do
  for r in $res; do
    timeout -k 10 240 python bench.py --no-cpu --no-single --no-match --no-sequence --groups $g --cu-reserve $r \
      --steps 20 --warmup 5 > gpurun_out/cm_${tag}_${g}_${r}.log 2>&1 || { echo "FAIL g=$g r=$r"; tail -20 gpurun_out/cm_${tag}_${g}_${r}.log; exit 1; }
    python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('groups',$g,'reserve',$r,'frames/s',d['value'],'ms/step',d['ms_per_step'],'stages',d.get('stages_ms'))" gpurun_out/cm_${tag}_${g}_${r}.log | tee -a $out
  done
done
