#!/bin/bash
# sqrt-free Jacobi convergence test, c = 1 shortcut: phases, GPU suite, latency-leg A/B
set -o pipefail
mkdir -p gpurun_out
VO_HIP_LIB=$PWD/monocular_visual_odometry_va4mr_amd/_build/diag_pnpprof.so timeout -k 10 200 python -u tools/pnp_prof.py 60 > gpurun_out/r6h_pnp_phases.txt 2>&1 || { tail -5 gpurun_out/r6h_pnp_phases.txt; exit 1; }
tail -1 gpurun_out/r6h_pnp_phases.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6h_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r6h_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r6h_gpu_tests.log
bash tools/gpu_seqab.sh r6h 2
