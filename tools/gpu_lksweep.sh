#!/bin/bash
# LK variant sweep: parity tests with the default kernel, then single-group stage times for
# k_lk_w (default) and k_lk_q at several blocks-per-chain.  usage: bash tools/gpu_lksweep.sh <tag>
tag=${1:-l}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1 || { tail -30 gpurun_out/pytest_$tag.log; exit 1; }
tail -2 gpurun_out/pytest_$tag.log
A="--stages --no-cpu --no-single --groups 1 --chains 192 --steps 10 --warmup 3"
VO_ONE_STREAM=1 timeout -k 10 200 python bench.py $A > /dev/null 2> gpurun_out/lkw_$tag.err || exit $?
echo "w: $(tail -1 gpurun_out/lkw_$tag.err)"
for nb in ${QNB:-64 128 256}; do
  VO_LK_QUAD=1 VO_LK_QNB=$nb VO_ONE_STREAM=1 timeout -k 10 200 python bench.py $A > /dev/null 2> gpurun_out/lkq${nb}_$tag.err || exit $?
  echo "q$nb: $(tail -1 gpurun_out/lkq${nb}_$tag.err)"
done
