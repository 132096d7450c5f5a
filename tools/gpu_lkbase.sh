#!/bin/bash
# k_lk_w baseline at the verdict's reference point (192 chains, one group, one stream):
# kernel-trace stats + the two SQ counter passes of tools/gpu_sq.sh.
# usage: bash tools/gpu_lkbase.sh <tag>
tag=${1:-lk}
mkdir -p gpurun_out
export TMPDIR=/tmp VO_ONE_STREAM=1
A="--no-cpu --no-single --no-match --no-sequence --groups 1 --chains 192 --steps 10 --warmup 3"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --kernel-include-regex "k_lk_w|k_pnp|k_gftt_select|k_eig3|k_pyr_level|k_triangulate|k_add_finish|k_track_compact" --output-format csv -d gpurun_out/kt_$tag -o run -- python bench.py $A > gpurun_out/kt_$tag.log 2>&1 || exit $?
rm -f gpurun_out/kt_$tag/*kernel_trace.csv
bash tools/gpu_sq.sh $tag --no-match --no-sequence --steps 4 || exit $?
python tools/sq_summary.py gpurun_out/sq1_$tag gpurun_out/sq2_$tag > gpurun_out/sq_$tag.txt
