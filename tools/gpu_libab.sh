#!/bin/bash
# A/B of two builds of libvo_hip.so on the headline bench (alternating, same box):
# usage: gpu_libab.sh <alt.so> [reps] [extra bench args]
mkdir -p gpurun_out
alt=$1; n=${2:-2}; shift 2
for i in $(seq $n); do for lib in default $alt; do
  if [ $lib = default ]; then unset VO_HIP_LIB; else export VO_HIP_LIB=$lib; fi
  timeout -k 10 200 python bench.py --no-cpu --no-single --no-match --no-sequence "$@" > gpurun_out/lab.json 2> gpurun_out/lab.err || { tail -5 gpurun_out/lab.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/lab.json').read().strip().splitlines()[-1]);print('$lib','fps',d['value'],'ms',d['ms_per_step'],'stages',d['stages_ms'])"
done; done
