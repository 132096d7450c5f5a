#!/bin/bash
# round-4: the new / changed GPU tests only (retain_best hook, SIFT capacity per chain,
# batched bootstrap workspace ownership, sequence cuts x stream groups)
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_retain_best.py \
  "tests/test_gpu_bootstrap.py::test_bootstrap_sift_capacity_marks_only_the_overflowing_chain" \
  "tests/test_gpu_bootstrap.py::test_batched_bootstrap_matches_oracle_per_chain" \
  tests/test_gpu_sequence.py -k "not full_sequence" > gpurun_out/r4tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r4tests.log | tail -30
exit $rc
