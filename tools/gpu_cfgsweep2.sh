#!/bin/bash
# (chains, groups, one-stream) sweep of the default bench step.  usage: bash tools/gpu_cfgsweep2.sh "384 2 0" "384 4 1" ...
mkdir -p gpurun_out
export TMPDIR=/tmp
for cg in "$@"; do
  set -- $cg
  VO_ONE_STREAM=$3 timeout -k 10 200 python bench.py --no-cpu --no-single --no-match --chains $1 --groups $2 --steps 20 --warmup 5 \
      > gpurun_out/cfg2.json 2> gpurun_out/cfg2.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/cfg2.json'));print('chains',$1,'groups',$2,'one_stream',$3,'fps',d['value'])"
done
