export TMPDIR=/tmp
O=gpurun_out; HL="--no-cpu --no-single --no-match --no-sequence"; KL="--kernel-include-regex k_lk_w"; R="--output-format csv"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VALU $KL $R -d $O/sq3_r6m -o run -- python bench.py $HL --steps 10 > $O/sq3_r6m.json 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_SMEM SQ_INSTS_VMEM_RD SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_THREAD_CYCLES_VALU $KL $R -d $O/sq4_r6m -o run -- python bench.py $HL --steps 10 > $O/sq4_r6m.json 2>&1 || exit $?
