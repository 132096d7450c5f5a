#!/bin/bash
# SQ instruction/stall counters for the step kernels (one --pmc pass each, own run).
# usage: bash tools/gpu_sq.sh <tag> [bench args...]
tag=${1:-s}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp VO_ONE_STREAM=1
A="--no-cpu --no-single --groups 1 --chains 192 --warmup 2 $@"
R="--kernel-include-regex k_lk_w|k_eig3|k_pyr_level|k_gftt_select|k_pnp_ransac --output-format csv"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY $R -d gpurun_out/sq1_$tag -o run -- python bench.py $A > gpurun_out/sq1_$tag.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE $R -d gpurun_out/sq2_$tag -o run -- python bench.py $A > gpurun_out/sq2_$tag.log 2>&1 || exit $?
