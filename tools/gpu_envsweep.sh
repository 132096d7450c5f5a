#!/bin/bash
# Stage times of the single-group bench under several environment settings (one bench run per
# setting, one stream).  usage: bash tools/gpu_envsweep.sh <tag> "ENV=a ENV2=b" "ENV=c" ...
tag=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
A="--stages --no-cpu --no-single --no-match --groups 1 --chains 192 --steps 10 --warmup 3"
i=0
for e in "$@"; do
  env VO_ONE_STREAM=1 $e timeout -k 10 200 python bench.py $A > /dev/null 2> gpurun_out/sweep_${tag}_$i.err || exit $?
  echo "[$e] $(tail -1 gpurun_out/sweep_${tag}_$i.err)"
  i=$((i+1))
done
