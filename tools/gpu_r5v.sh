#!/bin/bash
# round-5 verification: smoke(), the whole GPU suite, then a kernel-trace profile of the default bench
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5v_smoke.log 2>&1 || { tail -20 gpurun_out/r5v_smoke.log; exit 1; }
tail -1 gpurun_out/r5v_smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5v_tests.log 2>&1
rc=$?; grep -E "FAIL|ERROR|passed|failed" gpurun_out/r5v_tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
