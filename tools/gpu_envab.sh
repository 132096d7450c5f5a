#!/bin/bash
# A/B of one environment variable on the headline bench: usage gpu_envab.sh VAR v1 v2 [reps]
mkdir -p gpurun_out
var=$1; a=$2; b=$3; n=${4:-2}
for i in $(seq $n); do for v in $a $b; do
  env $var=$v timeout -k 10 200 python bench.py --no-cpu --no-single --no-match > gpurun_out/ab.json 2> gpurun_out/ab.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$var=$v','fps',d['value'],'track_ms',d['stages_ms']['track'])"
done; done
