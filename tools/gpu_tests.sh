#!/bin/bash
# the full GPU suite and the single-chain leg (no bench).  usage: gpu_tests.sh <tag>
set -e
tag=${1:-a}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_${tag}.log 2>&1 || true
timeout -k 10 200 python -u tools/single_prof.py 200 > gpurun_out/single_${tag}.log 2>&1
