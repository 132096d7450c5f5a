#!/bin/bash
# pyramid lookahead A/B: parity test, then the headline bench without / with lookahead
# (VO_LA_STREAM=own: the lookahead pyramid on a stream of its own)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_lookahead.py -x -q --timeout 200 --timeout-method thread > gpurun_out/la_t.log 2>&1 || { tail -30 gpurun_out/la_t.log; exit 1; }
tail -1 gpurun_out/la_t.log
for cfg in "0 side" "1 own" "0 side" "1 own"; do
  set -- $cfg
  VO_LA_STREAM=$2 timeout -k 10 200 python bench.py --no-cpu --no-single --no-match --no-sequence --lookahead $1 > gpurun_out/la.json 2> gpurun_out/la.err || { tail -5 gpurun_out/la.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/la.json').read().strip().splitlines()[-1]);print('la $cfg','fps',d['value'],'ms',d['ms_per_step'],'ok',d['chains_ok'],'stages',d['stages_ms'])"
done
