#!/bin/bash
# round-5: eig3 row loop unrolled + NMS maxima cached -- GFTT tests, solo kernel times for both builds, headline A/B
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
BASE=$PWD/monocular_visual_odometry_va4mr_amd/_build/libvo_base.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py -k "gftt or step or harris" > gpurun_out/r5y_tests.log 2>&1 || { tail -30 gpurun_out/r5y_tests.log; exit 1; }
tail -1 gpurun_out/r5y_tests.log
for lib in new base; do
  if [ $lib = base ]; then export VO_HIP_LIB=$BASE; else unset VO_HIP_LIB; fi
  VO_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/solo_$lib -o run -- python bench.py --groups 1 --chains 384 --no-sequence --no-single --no-match --no-cpu --steps 10 --warmup 3 > gpurun_out/solo_$lib.log 2>&1 || { tail -5 gpurun_out/solo_$lib.log; exit 1; }
  python tools/trace_by_grid.py gpurun_out/solo_$lib gpurun_out/solo_$lib/by_grid.csv && rm -f gpurun_out/solo_$lib/*kernel_trace.csv
  echo $lib; grep -E "k_eig3|k_lk_w" gpurun_out/solo_$lib/by_grid.csv | head -3
done
unset VO_HIP_LIB
bash tools/gpu_ab.sh r5y 2
