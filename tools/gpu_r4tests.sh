#!/bin/bash
# round-4: the whole GPU test suite (LK kernel changed; new retain_best / capacity / sequence
# cut tests)
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4tests.log 2>&1
rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/r4tests.log | tail -15
exit $rc
