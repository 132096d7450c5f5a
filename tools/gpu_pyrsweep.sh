#!/bin/bash
# k_pyr_level durations for VO_PYR_TH1 variants (single group, one stream)
mkdir -p gpurun_out
export TMPDIR=/tmp VO_ONE_STREAM=1
for th in "$@"; do
  VO_PYR_TH1=$th timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_pyr$th -o run -- python bench.py --no-cpu --no-single --no-match --groups 1 --chains 192 --steps 4 --warmup 2 > gpurun_out/kt_pyr$th.log 2>&1 || exit $?
  echo "TH1=$th"; python3 tools/trace_by_grid.py gpurun_out/kt_pyr$th gpurun_out/kt_pyr$th.csv && grep pyr_level gpurun_out/kt_pyr$th.csv
  rm -f gpurun_out/kt_pyr$th/*kernel_trace.csv
done
