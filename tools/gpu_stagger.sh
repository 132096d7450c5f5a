#!/bin/bash
# headline bench with and without the staggered group start
mkdir -p gpurun_out
for st in 0 1 0 1; do
  timeout -k 10 200 python bench.py --no-cpu --no-single --no-match --stagger $st "$@" > gpurun_out/stg.json 2> gpurun_out/stg.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/stg.json'));print('stagger',$st,'fps',d['value'])"
done
