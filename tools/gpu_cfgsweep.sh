#!/bin/bash
# Whole-step throughput of bench.py for several (chains, groups) configurations (two streams
# per GPU as in the default run).  usage: bash tools/gpu_cfgsweep.sh <tag> "384 2" "576 3" ...
tag=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for cg in "$@"; do
  set -- $cg
  timeout -k 10 300 python bench.py --no-cpu --no-single --no-match --chains $1 --groups $2 --steps 20 --warmup 5 \
      > gpurun_out/cfg_${tag}_$i.json 2> gpurun_out/cfg_${tag}_$i.err || exit $?
  python -c "import json,sys;d=json.load(open('gpurun_out/cfg_${tag}_$i.json'));print('chains',$1,'groups',$2,'fps',d['value'],'ms/step',d['ms_per_step'])"
  i=$((i+1))
done
