#!/bin/bash
# parallel-modulo subsets + 4-point epilogue: GPU tests, PnP profile, single chain and headline
# A/B against a first hypothesis round of 16 (libvo_hip_ch16.so).  usage: gpu_ransac2.sh <tag>
tag=${1:-a}
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ransac2_${tag}_pytest.txt 2>&1 || { tail -30 gpurun_out/ransac2_${tag}_pytest.txt; exit 1; }
tail -3 gpurun_out/ransac2_${tag}_pytest.txt
timeout -k 10 120 python -u tools/pnp_prof.py 80 > gpurun_out/ransac2_${tag}_pnp.log 2>&1 || exit 1
tail -2 gpurun_out/ransac2_${tag}_pnp.log
CH=$PWD/monocular_visual_odometry_va4mr_amd/_build/libvo_hip_ch16.so
for v in 1 2; do
  echo "default"; timeout -k 10 200 python -u tools/single_prof.py 200 2>&1 | grep frames
  echo "ch16"; VO_HIP_LIB=$CH timeout -k 10 200 python -u tools/single_prof.py 200 2>&1 | grep frames
done
for v in 1 2; do
  echo "default"; timeout -k 10 300 python -u bench.py --no-cpu --no-single --no-match --no-sequence --steps 30 --warmup 5 2>&1 | tail -1 | cut -c1-200
  echo "ch16"; VO_HIP_LIB=$CH timeout -k 10 300 python -u bench.py --no-cpu --no-single --no-match --no-sequence --steps 30 --warmup 5 2>&1 | tail -1 | cut -c1-200
done
