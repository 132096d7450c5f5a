#!/bin/bash
# k_lk_w time at 192 chains (one group, one stream), kernel-trace stats only, plus the LK
# bit-exact tests.  usage: bash tools/gpu_lkquick.sh <tag>
tag=${1:-q}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k "lk or step_parity" tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/lkq_$tag.log 2>&1 || { tail -20 gpurun_out/lkq_$tag.log; exit 1; }
tail -1 gpurun_out/lkq_$tag.log
VO_ONE_STREAM=1 timeout -s KILL 200 rocprofv3 --kernel-trace --stats --kernel-include-regex "k_lk_w" --output-format csv -d gpurun_out/kt_$tag -o run -- python bench.py --no-cpu --no-single --no-match --no-sequence --groups 1 --chains 192 --steps 10 --warmup 3 > gpurun_out/kt_$tag.log 2>&1 || exit $?
rm -f gpurun_out/kt_$tag/*kernel_trace.csv
grep k_lk_w gpurun_out/kt_$tag/run_kernel_stats.csv | cut -d, -f2-7
python -c "import json;d=json.load(open('gpurun_out/kt_$tag.log'));print('frames/s',d['value'],'points',d['points_last_step'],'track_ms',d['stages_ms']['track'])" 2>/dev/null || tail -2 gpurun_out/kt_$tag.log
