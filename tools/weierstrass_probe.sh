#!/bin/bash
# How many of OpenCV's 300 solvePoly sweeps the five-point solves run (CPU, oracle build):
# every degree-10 polynomial the oracle's findEssentialMat solves is captured (a hook inserted
# into a /tmp copy of oracle/vo_oracle_geom.c) and re-run with bit-exact cycle detection.
#   bash tools/weierstrass_probe.sh            synthetic matches (20 problems, 30 % outliers)
#   bash tools/weierstrass_probe.sh real       the C2 bootstrap matches of 6 shard starts
#                                              (tools/dump_boot_matches.py, oracle pipeline)
#   bash tools/weierstrass_probe.sh pipe       k_essential's 10-lane pipelined sweep schedule
#                                              (five_point_grp), emulated on the CPU, against
#                                              the oracle's serial solve_poly, bit for bit
set -e
mkdir -p /tmp/wk
R=$(cd "$(dirname "$0")/.." && pwd)
sed 's|int nroots = solve_poly(coeffs, 10, roots);|int nroots = solve_poly(coeffs, 10, roots); sp_hook(coeffs);|' "$R/oracle/vo_oracle_geom.c" > /tmp/wk/geom_hooked.c
cp "$R/tools/micro/weierstrass_probe.c" /tmp/wk/
gcc -O2 -ffp-contract=off -fno-fast-math -std=gnu11 -I"$R/oracle" -I"$R/monocular_visual_odometry_va4mr_amd/csrc" \
    /tmp/wk/weierstrass_probe.c "$R/oracle/vo_oracle_img.c" -o /tmp/wk/probe -lm
if [ "$1" = pipe ]; then
  cp "$R/tools/micro/weierstrass_pipe_check.c" /tmp/wk/
  gcc -O2 -ffp-contract=off -fno-fast-math -std=gnu11 -I"$R/oracle" -I"$R/monocular_visual_odometry_va4mr_amd/csrc" \
      -I/tmp/wk /tmp/wk/weierstrass_pipe_check.c "$R/oracle/vo_oracle_img.c" -o /tmp/wk/pipe_check -lm
  /tmp/wk/pipe_check
  exit 0
fi
if [ "$1" = real ]; then
  python3 "$R/tools/dump_boot_matches.py" 0 700 1400 2100 2800 3500
  python3 -c "
import numpy as np
z = np.load('/tmp/wk/matches.npz')
for i in range(6):
    np.concatenate([z[f'p0_{i}'], z[f'p1_{i}']], 1).astype(np.float32).tofile(f'/tmp/wk/m_{i}.bin')"
  /tmp/wk/probe 6 0 file
else
  /tmp/wk/probe 20 0.3
fi
