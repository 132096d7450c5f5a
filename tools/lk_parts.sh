#!/bin/bash
# k_lk_w cost attribution: the same saved points tracked by the normal build and by builds with
# one part of the per-level fixed work removed (make -C monocular_visual_odometry_va4mr_amd/csrc lkx, then
# copy each _build/libvo_hip_lkx_<V>.so to _build/libvo_lkx_<V>.so: .gpurunignore drops libvo_hip_*.so)
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/lkx
timeout -k 10 200 python -u tools/lk_iter_cost.py --save gpurun_out/lkx 16 384 > gpurun_out/lkx/base.jsonl 2> gpurun_out/lkx/err.txt || { tail -5 gpurun_out/lkx/err.txt; exit 1; }
for rep in 1 2; do
for v in "" NOQT NOSTAGE NOTENSOR NOERR; do
  if [ -n "$v" ]; then lib=monocular_visual_odometry_va4mr_amd/_build/libvo_lkx_$v.so; else lib=monocular_visual_odometry_va4mr_amd/_build/libvo_hip.so; fi
  VO_HIP_LIB=$PWD/$lib timeout -k 10 200 python -u tools/lk_iter_cost.py --load gpurun_out/lkx 16 384 2>> gpurun_out/lkx/err.txt | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('${v:-BASE}', d['B'], d['points'], [(r['count'], r['ms']) for r in d['runs']])" || exit 1
done
done
rm -f gpurun_out/lkx/*.npz
