#!/bin/bash
# BF 2-NN matcher: parity tests, int8 vs bf16 A/B on the C5 / C3 legs, and the kernel trace +
# SQ counters of the int8 kernel alone at C5 size (tools/gpu_bfprof.sh).  usage: gpu_bf.sh <tag>
set -e
tag=${1:-a}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "bf_knn2 or sift or bootstrap_matches" > gpurun_out/pytest_bf_${tag}.log 2>&1
timeout -k 10 400 python -u tools/bf_ab.py > gpurun_out/bf_ab_${tag}.log 2>&1
bash tools/gpu_bfprof.sh $tag
