#!/bin/bash
# round-5: SQ counters of k_eig3 and k_gftt_select at the headline (two passes, each its own run)
export TMPDIR=/tmp
mkdir -p gpurun_out
H="--no-cpu --no-single --no-match --no-sequence --steps 10 --warmup 3"
KL="--kernel-include-regex k_eig3|k_gftt_select|k_pnp_tri"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY $KL --output-format csv -d gpurun_out/eq1 -o run -- python bench.py $H > gpurun_out/eq1.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE $KL --output-format csv -d gpurun_out/eq2 -o run -- python bench.py $H > gpurun_out/eq2.log 2>&1 || exit $?
python3 tools/sq_summary.py gpurun_out/eq1 gpurun_out/eq2 > gpurun_out/r5x_sq.txt 2>&1; cat gpurun_out/r5x_sq.txt
rm -rf gpurun_out/eq1 gpurun_out/eq2
