#!/bin/bash
# round-5: headline vs hardware queues per process (4 / 8 / 16 / 32), and the kernel timeline at 16
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
out=gpurun_out/r5e_hwq.jsonl; : > $out
hl() { local q=$1; timeout -k 10 200 python -u bench.py --no-sequence --no-single --no-match --no-cpu --steps 20 --warmup 5 --hw-queues $q > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; return 1; }
  tail -1 gpurun_out/ab.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print(json.dumps({'hwq': $q, 'value': d['value'], 'ms': d['ms_per_step'], 'ok': d['chains_ok']}))" | tee -a $out; }
hl 8 && hl 16 && hl 32 && hl 4 && hl 8 && hl 16 && hl 32 || exit 1
GPU_MAX_HW_QUEUES=16 bash tools/gpu_timeline.sh r5q16 > /dev/null 2>&1 || exit 1
sed -n '50,100p' gpurun_out/tl_r5q16.txt
