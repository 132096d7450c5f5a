#!/bin/bash
# Round-2 profile set of the default bench (summarised locally by prof_summary.py and
# valu_summary.py into profiles/): kernel-trace stats of the full default run, FETCH_SIZE /
# WRITE_SIZE passes and two SQ passes of the headline workload only (each its own run).
# usage: bash tools/gpu_prof_r2.sh <tag>
tag=${1:-r2}
mkdir -p gpurun_out
export TMPDIR=/tmp
H="--no-cpu --no-single --no-match --no-sequence"
R="--output-format csv"
K="--kernel-include-regex ::k_"
timeout -k 10 400 rocprofv3 --kernel-trace --stats $R -d gpurun_out/prof_$tag -o run -- python bench.py > gpurun_out/prof_$tag.json 2> gpurun_out/prof_$tag.err || exit $?
python3 tools/trace_by_grid.py gpurun_out/prof_$tag gpurun_out/prof_${tag}_by_grid.csv
rm -f gpurun_out/prof_$tag/*kernel_trace.csv
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE $K $R -d gpurun_out/pmc_fetch_$tag -o run -- python bench.py $H > gpurun_out/pmc_fetch_$tag.json 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE $K $R -d gpurun_out/pmc_write_$tag -o run -- python bench.py $H > gpurun_out/pmc_write_$tag.json 2>&1 || exit $?
KL="--kernel-include-regex k_lk_w"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY $KL $R -d gpurun_out/sq1_$tag -o run -- python bench.py $H > gpurun_out/sq1_$tag.json 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE $KL $R -d gpurun_out/sq2_$tag -o run -- python bench.py $H > gpurun_out/sq2_$tag.json 2>&1 || exit $?
du -sh gpurun_out/*_$tag*
