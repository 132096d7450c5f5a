#!/bin/bash
# LK kernel A/B on SQ counters and kernel time: k_lk_h (VO_LK_HALF=1) vs k_lk_w (0), one
# stream, 192 chains (no overlap with other stages), each counter set in its own run.
# usage: bash tools/gpu_lksq.sh <tag>
tag=${1:-q}
mkdir -p gpurun_out
export TMPDIR=/tmp VO_ONE_STREAM=1
A="--no-cpu --no-single --no-match --no-sequence --groups 1 --chains 192 --warmup 2 --steps 6"
R="--kernel-include-regex k_lk_ --output-format csv"
for h in 1 0; do
  export VO_LK_HALF=$h
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats $R -d gpurun_out/lksq_${tag}_t$h -o run -- python bench.py $A > gpurun_out/lksq_${tag}_t$h.log 2>&1 || exit $?
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY $R -d gpurun_out/lksq_${tag}_a$h -o run -- python bench.py $A > gpurun_out/lksq_${tag}_a$h.log 2>&1 || exit $?
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE $R -d gpurun_out/lksq_${tag}_b$h -o run -- python bench.py $A > gpurun_out/lksq_${tag}_b$h.log 2>&1 || exit $?
  echo "half=$h"; python tools/sq_summary.py gpurun_out/lksq_${tag}_a$h gpurun_out/lksq_${tag}_b$h
  grep -h "k_lk" gpurun_out/lksq_${tag}_t$h/*kernel_stats.csv | cut -c1-200
done
