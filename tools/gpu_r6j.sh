#!/bin/bash
# pyramid tail for 9..64 chains: parity + sequence tests, latency-leg A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sequence.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6j_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r6j_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r6j_gpu_tests.log
bash tools/gpu_seqab.sh r6j 2
