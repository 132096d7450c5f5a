#!/bin/bash
# E-RANSAC cost attribution: k_essential average time in a 64-chain bootstrap (tools/boot_prof.py)
# for libvo_hip.so and the -DVO_ESSX_* timing builds (make -C .../csrc ../_build/libvo_hip_essx_X.so)
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/essx
for lib in libvo_hip.so "$@"; do
    d=gpurun_out/essx/${lib%.so}
    rm -rf "$d"
    VO_HIP_LIB=$PWD/monocular_visual_odometry_va4mr_amd/_build/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o p -- python -u tools/boot_prof.py 64 > "$d.log" 2>&1 || { tail -5 "$d.log"; exit 1; }
    f=$(find "$d" -name "*kernel_stats.csv" | head -1)
    echo "$lib: $(grep -h 'k_essential' "$f" | awk -F, '{printf "%s calls avg %.1f us ", $2, $4/1000}')"
    find "$d" -name "*kernel_trace.csv" -delete
done
