#!/bin/bash
# stream-priority variants of the default bench step.  usage: bash tools/gpu_priosweep.sh none g0 side
mkdir -p gpurun_out
for p in "$@"; do
  timeout -k 10 200 python bench.py --no-cpu --no-single --no-match --prio $p --steps 30 --warmup 5 > gpurun_out/prio.json 2> gpurun_out/prio.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/prio.json'));print('prio','$p','fps',d['value'])"
done
