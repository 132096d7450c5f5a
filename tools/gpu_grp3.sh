#!/bin/bash
# headline configuration sweep: stream groups x chains per GPU (alternating)
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "2 768" "3 768" "2 1024" "3 1152" "2 768"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --no-cpu --no-single --no-match --no-sequence --groups $1 --chains $2 > gpurun_out/g3.json 2> gpurun_out/g3.err || { tail -5 gpurun_out/g3.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/g3.json').read().strip().splitlines()[-1]);print('groups $1 chains $2','fps',d['value'],'ms',d['ms_per_step'],'ok',d['chains_ok'])"
done
