#!/bin/bash
# SIFT kernels of the batched bootstrap (tools/sift_bench.py, KITTI): kernel-trace stats and
# SQ counters (two --pmc passes, each its own run).  usage: bash tools/gpu_sift_sq.sh <tag>
tag=${1:-s}
mkdir -p gpurun_out
export TMPDIR=/tmp
R="--kernel-include-regex k_sift_desc_w|k_extrema|k_blur_tile|k_sift_ori|k_sift_refine --output-format csv"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats $R -d gpurun_out/sk_$tag -o run -- python tools/sift_bench.py 3 kitti > gpurun_out/sk_$tag.log 2>&1 || exit $?
python tools/trace_by_grid.py gpurun_out/sk_$tag gpurun_out/sk_$tag/by_grid.csv; rm -f gpurun_out/sk_$tag/*kernel_trace.csv
[ "$2" = "stats" ] && { head -30 gpurun_out/sk_$tag/by_grid.csv; exit 0; }
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY $R -d gpurun_out/ss1_$tag -o run -- python tools/sift_bench.py 1 kitti > gpurun_out/ss1_$tag.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE $R -d gpurun_out/ss2_$tag -o run -- python tools/sift_bench.py 1 kitti > gpurun_out/ss2_$tag.log 2>&1 || exit $?
cat gpurun_out/sk_$tag.log
