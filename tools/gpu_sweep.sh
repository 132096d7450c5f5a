#!/bin/bash
# bench sweep over chains-per-GPU x stream groups; usage: bash tools/gpu_sweep.sh tag "B:G B:G ..."
tag=$1; shift
mkdir -p gpurun_out
for bg in $1; do
  b=${bg%:*}; g=${bg#*:}
  timeout -k 10 300 python bench.py --no-cpu --no-single --chains $b --groups $g --steps 20 > gpurun_out/sweep_${tag}_${b}_${g}.json 2>gpurun_out/sweep_${tag}_${b}_${g}.err || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/sweep_${tag}_${b}_${g}.json')); print('B=$b G=$g', d['value'], d['ms_per_step'], d.get('host_ms_per_step'), d['stages_ms'], d['chain_status'])"
done
