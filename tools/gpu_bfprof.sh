#!/bin/bash
# k_bf_i8 alone (tools/bf_micro.py): kernel trace + SQ counter passes.  usage: gpu_bfprof.sh <tag>
tag=${1:-a}
mkdir -p gpurun_out
export TMPDIR=/tmp
P="python3 tools/bf_micro.py 10"
timeout -k 10 120 $P > gpurun_out/bfp_${tag}.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bfp_${tag}_t -o run -- $P >> gpurun_out/bfp_${tag}.log 2>&1 || exit $?
R="--kernel-include-regex k_bf_i8 --output-format csv"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY $R -d gpurun_out/bfp_${tag}_a -o run -- $P > /dev/null 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE $R -d gpurun_out/bfp_${tag}_b -o run -- $P > /dev/null 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD $R -d gpurun_out/bfp_${tag}_c -o run -- $P > /dev/null 2>&1 || true
python3 tools/sq_summary.py gpurun_out/bfp_${tag}_a gpurun_out/bfp_${tag}_b gpurun_out/bfp_${tag}_c >> gpurun_out/bfp_${tag}.log
grep -h "k_bf" gpurun_out/bfp_${tag}_t/*kernel_stats.csv | cut -c1-160 >> gpurun_out/bfp_${tag}.log
