#!/bin/bash
# A/B of SIFT builds: for each library, the SIFT parity tests (oracle, wave == serial) and the
# batched per-image time (sift_bench, KITTI batch 64).
# usage: bash tools/gpu_siftab.sh <tag> <lib.so> [<lib.so> ...]   ("default" = _build/libvo_hip.so)
tag=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in "$@"; do
  if [ "$lib" = default ]; then unset VO_HIP_LIB; else export VO_HIP_LIB=$PWD/$lib; fi
  echo "== $lib"
  timeout -k 10 300 python -u -m pytest tests/test_gpu_bootstrap.py -x -q --timeout 200 --timeout-method thread \
      -k "sift or batched_bootstrap" > gpurun_out/siftab_${tag}_t.log 2>&1 || { tail -20 gpurun_out/siftab_${tag}_t.log; exit 1; }
  tail -1 gpurun_out/siftab_${tag}_t.log
  timeout -k 10 200 python tools/sift_bench.py 6 kitti,malaga1024 || exit 1
done
