#!/bin/bash
# Headline bench (no side legs) over stream-group counts: usage gpu_grpsw.sh "2 3 4" [reps]
mkdir -p gpurun_out
for i in $(seq ${2:-1}); do for g in $1; do
  timeout -k 10 200 python bench.py --no-cpu --no-single --no-match --no-sequence --groups $g > gpurun_out/gs.json 2> gpurun_out/gs.err || { tail -5 gpurun_out/gs.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/gs.json').read().strip().splitlines()[-1]);print('groups $g','fps',d['value'],'ms',d['ms_per_step'],'boot',d['bootstrap_s'])"
done; done
