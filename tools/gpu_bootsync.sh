#!/bin/bash
# bootstrap without the host synchronisation (SIFT capacity folded into the chain status):
# GPU tests, then the 768-chain bootstrap time.  usage: gpu_bootsync.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/bootsync_pytest.txt 2>&1 || { tail -20 gpurun_out/bootsync_pytest.txt; exit 1; }
tail -1 gpurun_out/bootsync_pytest.txt
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --no-cpu --no-single --no-match --no-sequence --steps 3 --warmup 1 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['bootstrap_s'], d['value'], d['chains_ok'])" || exit 1
done
