#!/bin/bash
# k_add_finish as a 4-wave, 16 KB-LDS block: GPU suite, latency-leg + headline A/B, C5 A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6l_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r6l_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r6l_gpu_tests.log
bash tools/gpu_seqab.sh r6l 2 || exit 1
BASE=$PWD/monocular_visual_odometry_va4mr_amd/_build/libvo_base.so
for i in 1 2; do
  timeout -k 10 300 python -u tools/c5_only.py 256 2 > gpurun_out/r6l_c5_new_$i.txt 2>&1 && tail -1 gpurun_out/r6l_c5_new_$i.txt || exit 1
  VO_HIP_LIB=$BASE timeout -k 10 300 python -u tools/c5_only.py 256 2 > gpurun_out/r6l_c5_base_$i.txt 2>&1 && tail -1 gpurun_out/r6l_c5_base_$i.txt || exit 1
done
