#!/bin/bash
# round-4 probe 3: headline step with the latency stages on a high-priority stream and/or more
# hardware queues per process (A/B, alternating)
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for rep in 1 2; do
for cfg in "0 4" "1 4" "0 8" "1 8"; do
  set -- $cfg
  VO_PRIO_LATENCY=$1 timeout -k 10 200 python -u bench.py --no-cpu --no-single --no-match --no-sequence --steps 20 --warmup 5 --hw-queues $2 > gpurun_out/p3_$1_$2.json 2> gpurun_out/p3.err || { tail -5 gpurun_out/p3.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/p3_$1_$2.json').read().splitlines()[-1])
print('prio $1 queues $2', d['value'], d['ms_per_step'], d['chains_ok'], d['stages_ms'])"
done
done
