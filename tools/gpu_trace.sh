#!/bin/bash
# per-dispatch kernel trace (kept) + SQ counters for kernels matching a regex
# usage: bash tools/gpu_trace.sh <tag> <regex>
tag=${1:-t}; rx=${2:-k_pyr_level}
mkdir -p gpurun_out
export TMPDIR=/tmp VO_ONE_STREAM=1
A="--no-cpu --no-single --groups 1 --chains 192 --steps 4 --warmup 2"
R="--kernel-include-regex $rx --output-format csv"
timeout -k 10 300 rocprofv3 --kernel-trace $R -d gpurun_out/tr_$tag -o run -- python bench.py $A > gpurun_out/tr_$tag.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY $R -d gpurun_out/sqt1_$tag -o run -- python bench.py $A > gpurun_out/sqt1_$tag.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE $R -d gpurun_out/sqt2_$tag -o run -- python bench.py $A > gpurun_out/sqt2_$tag.log 2>&1 || exit $?
