#!/bin/bash
# Headline bench (no side legs) for each value of one environment variable, repeated:
# usage: gpu_envsw.sh VAR "v1 v2 ..." [reps] [extra bench args]
mkdir -p gpurun_out
var=$1; vals=$2; n=${3:-1}; shift 3
for i in $(seq $n); do for v in $vals; do
  env $var=$v timeout -k 10 200 python bench.py --no-cpu --no-single --no-match --no-sequence "$@" > gpurun_out/sw.json 2> gpurun_out/sw.err || { tail -5 gpurun_out/sw.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1]);print('$var=$v','fps',d['value'],'ms',d['ms_per_step'],'stages',d['stages_ms'])"
done; done
