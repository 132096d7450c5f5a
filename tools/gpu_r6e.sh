#!/bin/bash
# fp64 dependent-op latencies; PnP phases with 32 / 16 / 8 first-round hypotheses
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 tools/micro/f64_latency > gpurun_out/r6e_f64_latency.txt 2>&1 || { cat gpurun_out/r6e_f64_latency.txt; exit 1; }
cat gpurun_out/r6e_f64_latency.txt
for v in "" _ch16 _ch8; do
  VO_HIP_LIB=$PWD/monocular_visual_odometry_va4mr_amd/_build/diag_pnpprof$v.so timeout -k 10 200 python -u tools/pnp_prof.py 60 > gpurun_out/r6e_pnp$v.txt 2>&1 || { tail -5 gpurun_out/r6e_pnp$v.txt; exit 1; }
  echo "== $v"; tail -1 gpurun_out/r6e_pnp$v.txt
done
