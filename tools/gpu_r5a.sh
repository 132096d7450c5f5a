#!/bin/bash
# round-5: LGKM counter probe, headline-shape reference check of the product library and of the
# dropped k_lk_w variant (libvo_lkvar.so), the LK parity + new / re-parametrised GPU tests, bench
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 60 ./tools/micro/lgkm_probe 8192 64 > gpurun_out/r5_lgkm_probe.txt 2>&1 || { cat gpurun_out/r5_lgkm_probe.txt; exit 1; }
cat gpurun_out/r5_lgkm_probe.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r5a_lk_tests.log 2>&1
rc=$?; grep -E "FAIL|ERROR|passed|failed" gpurun_out/r5a_lk_tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u tools/lk_variant_probe.py --steps 25 > gpurun_out/r5_probe_product.json 2> gpurun_out/r5_probe_product.err || { tail -5 gpurun_out/r5_probe_product.err; exit 1; }
cut -c1-600 gpurun_out/r5_probe_product.json
VO_HIP_LIB=$PWD/monocular_visual_odometry_va4mr_amd/_build/libvo_lkvar.so timeout -k 10 300 python -u tools/lk_variant_probe.py --steps 25 --detail > gpurun_out/r5_probe_lkvar.json 2> gpurun_out/r5_probe_lkvar.err || { tail -5 gpurun_out/r5_probe_lkvar.err; exit 1; }
cut -c1-1500 gpurun_out/r5_probe_lkvar.json
timeout -k 10 500 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_step_paths.py tests/test_gpu_bootstrap.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r5a_tests.log 2>&1
rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/r5a_tests.log | tail -15
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_r4bench.sh r5a
