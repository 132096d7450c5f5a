#!/bin/bash
# final tree: full GPU suite + smoke
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r6p_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r6p_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r6p_gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6p_smoke.log 2>&1 || { tail -20 gpurun_out/r6p_smoke.log; exit 1; }
tail -1 gpurun_out/r6p_smoke.log
