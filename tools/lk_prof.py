#!/usr/bin/env python3
"""Per-block timings of the LK level kernels for one chain (diagnostics build).

    make -C monocular_visual_odometry_va4mr_amd/csrc ../_build/libvo_hip_lkprof.so
    python tools/lk_prof.py [n_frames]

Runs the drop-in class eagerly on KITTI-size synthetic frames with the VO_LK_PROF library
and reports, for the last frame's tracking step, each level's span (first block start to
last block end), block durations, LK iterations and J-tile stagings per block."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["VO_HIP_LIB"] = os.path.join(ROOT, "monocular_visual_odometry_va4mr_amd", "_build", "libvo_hip_lkprof.so")
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from monocular_visual_odometry_va4mr_amd import _lib as L  # noqa: E402
from monocular_visual_odometry_va4mr_amd import options as Op  # noqa: E402
from monocular_visual_odometry_va4mr_amd.synth import Renderer, poses  # noqa: E402
from monocular_visual_odometry_va4mr_amd.VisualOdometryPipeLine import VisualOdometryPipeLine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
rend = Renderer("kitti", seed=1, device="cuda")
Rs, cs = poses(n, rend.p)
fr = rend.render_batch(list(range(n)), Rs, cs)
opts, boot, _ = Op.get("kitti")
vo = VisualOdometryPipeLine(rend.K, opts, max_frames=n + 8, use_graph=False)
vo.initialization(fr[boot[0]], fr[boot[1]])
for i in range(boot[1] + 1, n):
    vo.continuous_operation(fr[i])
torch.cuda.synchronize()
buf = np.zeros((L.VO_MAX_LEVELS, 1024, 8), np.int64)
lib = L.lib()
lib.vo_lk_prof_read.restype = C.c_int
assert lib.vo_lk_prof_read(C.c_void_p(buf.ctypes.data)) == 0
eng = vo._eng
npts = int(eng.t["nL"][0]) + int(eng.t["nC"][0])
print(f"points after tracking: {npts} (landmarks {int(eng.t['nL'][0])}, candidates {int(eng.t['nC'][0])})")
t0 = buf[:, :, 0][buf[:, :, 0] > 0].min()
for lv in range(eng.dims.nlev - 1, -1, -1):
    b = buf[lv]
    used = b[:, 1] > 0
    ph = b[:npts, 4:8].mean(0) / 100.0
    phases = f"phases us/point: I-stage {ph[0]:5.2f} tensor {ph[1]:5.2f} J-stage {ph[2]:5.2f} iterations(+restage) {ph[3]:5.2f}"
    if not used.any():      # fused launch: only level 0 holds the block times
        it = b[:npts, 2]
        print(f"level {lv}: iters mean {it.mean():5.2f} max {it.max():3d} | {phases}")
        continue
    st, en = b[used, 0], b[used, 1]
    dur = (en - st) / 100.0
    it, sg = b[used, 2], b[used, 3]
    k = int(np.argmax(dur))
    print(f"level {lv}: blocks {used.sum():4d}  span {(en.max() - st.min()) / 100.0:6.1f} us  start {(st.min() - t0) / 100.0:7.1f} "
          f"| block us mean {dur.mean():5.2f} p50 {np.median(dur):5.2f} p99 {np.percentile(dur, 99):6.2f} max {dur.max():6.2f} "
          f"| iters mean {it.mean():5.2f} max {it.max():3d} (slowest block: {it[k]} iters, {sg[k]} stagings) "
          f"| start spread {(st.max() - st.min()) / 100.0:5.1f} us")
    print("    " + phases)
