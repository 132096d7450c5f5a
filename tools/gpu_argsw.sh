#!/bin/bash
# Headline bench (no side legs) for several bench argument sets: usage gpu_argsw.sh "args1" "args2" ...
mkdir -p gpurun_out
for a in "$@"; do
  timeout -k 10 200 python bench.py --no-cpu --no-single --no-match --no-sequence $a > gpurun_out/as.json 2> gpurun_out/as.err || { tail -5 gpurun_out/as.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/as.json').read().strip().splitlines()[-1]);print('[$a]','fps',d['value'],'ms',d['ms_per_step'],'stages',d['stages_ms'])"
done
