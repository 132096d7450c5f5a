#!/bin/bash
# A/B library from another revision: compiles csrc/*.hip as of git revision <rev> into
# monocular_visual_odometry_va4mr_amd/_build/libvo_<name>.so (VO_HIP_LIB=... selects it at run time;
# the name must not match .gpurunignore's libvo_hip_*.so).  usage: tools/build_ab.sh <rev> <name>
set -e
rev=$1; name=$2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$root" archive "$rev" monocular_visual_odometry_va4mr_amd/csrc include | tar -x -C "$tmp"
make -s -j8 -C "$tmp/monocular_visual_odometry_va4mr_amd/csrc" ../_build/libvo_hip.so
cp "$tmp/monocular_visual_odometry_va4mr_amd/_build/libvo_hip.so" "$root/monocular_visual_odometry_va4mr_amd/_build/libvo_$name.so"
rm -rf "$tmp"
echo "$root/monocular_visual_odometry_va4mr_amd/_build/libvo_$name.so"
