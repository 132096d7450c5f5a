#!/bin/bash
# fused small-level pyramid (k_pyr_tail): GPU suite, latency-leg A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6i_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r6i_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r6i_gpu_tests.log
bash tools/gpu_seqab.sh r6i 2
