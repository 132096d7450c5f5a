#!/bin/bash
# Round-3 profile set of the default bench, in two GPU calls (each under the call's time limit):
#   bash tools/gpu_prof_r3.sh trace <tag>   kernel-trace stats of the full default run
#   bash tools/gpu_prof_r3.sh pmc <tag>     FETCH_SIZE / WRITE_SIZE passes and two k_lk_w SQ
#                                           passes of the headline workload only (each its own run)
# summarised locally by tools/prof_summary.py and tools/valu_summary.py into profiles/.
what=${1:-trace}
tag=${2:-r3}
mkdir -p gpurun_out
export TMPDIR=/tmp
H="--no-cpu --no-single --no-match --no-sequence"
R="--output-format csv"
K="--kernel-include-regex ::k_"
if [ "$what" = trace ]; then
  timeout -k 10 500 rocprofv3 --kernel-trace --stats $R -d gpurun_out/prof_$tag -o run -- python bench.py > gpurun_out/prof_$tag.json 2> gpurun_out/prof_$tag.err || exit $?
  python3 tools/trace_by_grid.py gpurun_out/prof_$tag gpurun_out/prof_${tag}_by_grid.csv
  rm -f gpurun_out/prof_$tag/*kernel_trace.csv
else
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE $K $R -d gpurun_out/pmc_fetch_$tag -o run -- python bench.py $H > gpurun_out/pmc_fetch_$tag.json 2>&1 || exit $?
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE $K $R -d gpurun_out/pmc_write_$tag -o run -- python bench.py $H > gpurun_out/pmc_write_$tag.json 2>&1 || exit $?
  KL="--kernel-include-regex k_lk_w"
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY $KL $R -d gpurun_out/sq1_$tag -o run -- python bench.py $H > gpurun_out/sq1_$tag.json 2>&1 || exit $?
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE $KL $R -d gpurun_out/sq2_$tag -o run -- python bench.py $H > gpurun_out/sq2_$tag.json 2>&1 || exit $?
fi
du -sh gpurun_out/*_$tag* | tail -8
