#!/bin/bash
# round-5: sequence plan sweep (rank slices, overlap 30 / 15 / 10) and the 15-frame GPU sequence tests
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/slice_sweep.py 1:64:30 1:64:15 1:64:10 1:48:15 1:96:15 8:32:30 8:32:15 8:32:10 8:16:15 8:24:15 8:48:15 4:32:15 2:32:15 > gpurun_out/r5_slice_sweep.jsonl 2> gpurun_out/r5_slice_sweep.err || { tail -5 gpurun_out/r5_slice_sweep.err; exit 1; }
cat gpurun_out/r5_slice_sweep.jsonl
timeout -k 10 400 python -u -m pytest tests/test_gpu_sequence.py -x -v --timeout 300 --timeout-method thread -k "15" > gpurun_out/r5c_tests.log 2>&1
rc=$?; grep -E "FAIL|ERROR|passed|failed" gpurun_out/r5c_tests.log | tail -6; exit $rc
