#!/bin/bash
# Targeted GPU tests first (fail fast on the newest kernels), then the round-end verification
# (full -m gpu suite, smoke, default bench line).  usage: bash tools/gpu_new.sh <tag> "<pytest -k expr>"
tag=${1:-n}
sel=${2:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$sel" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$sel" > gpurun_out/pytest_sel_$tag.log 2>&1
  rc=$?
  tail -3 gpurun_out/pytest_sel_$tag.log
  [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/pytest_sel_$tag.log | head -20; exit $rc; }
fi
bash tools/gpu_final.sh $tag
