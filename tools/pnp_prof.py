#!/usr/bin/env python3
"""Phase times of the fused PnP + triangulation launch (k_pnp_tri, block 0) for one KITTI chain
stepped like the drop-in class (one chain, eager).  Needs the diagnostics build
(make -C monocular_visual_odometry_va4mr_amd/csrc ../_build/libvo_hip_pnpprof.so).
usage: python tools/pnp_prof.py [n_frames]"""
import ctypes as C
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("VO_HIP_LIB", os.path.join(HERE, "monocular_visual_odometry_va4mr_amd", "_build", "libvo_hip_pnpprof.so"))
sys.path.insert(0, HERE)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from monocular_visual_odometry_va4mr_amd import _lib as L  # noqa: E402
from monocular_visual_odometry_va4mr_amd import options as Op  # noqa: E402
from monocular_visual_odometry_va4mr_amd.engine import Engine  # noqa: E402
from monocular_visual_odometry_va4mr_amd.synth import Renderer  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 60
dev = torch.device("cuda")
opts, (b0, b1), _ = Op.get("kitti")
gap = b1 - b0
rend = Renderer("kitti", seed=1, device=dev)
gt = bench.StagePoses(n + gap + 8, rend.p)
fr = bench.render_windows(rend, gt, [0], gap, n - 2, dev)[:, 0]
eng = Engine(rend.K, opts, fr.shape[-1], fr.shape[-2], batch=1, device=dev, ncap=16384, pcap=16384, fcap=n + 8)
eng.bootstrap(fr[0:1], fr[1:2])
lib = L.lib()
lib.vo_pnp_prof_read.argtypes = [C.c_void_p]
buf = (C.c_longlong * 32)()
names = [("ransac", 0, 3), ("r:prior rounds", 0, 1), ("r:subsets", 1, 6), ("r:p3p", 6, 2), ("r:score", 2, 3), ("s:score1", 2, 28), ("s:rule1", 28, 29), ("inl+compact", 3, 4), ("epnp prep", 4, 10), ("MtM", 10, 16), ("svd12", 16, 11), ("betas+Rt", 11, 13), ("b1:lsq", 11, 17), ("b1:gn", 17, 18),
         ("b2:lsq", 11, 24), ("b2:gn", 24, 25), ("b3:lsq", 11, 19), ("b3:gn", 19, 23),
         ("pick", 13, 5), ("apply", 5, 14), ("triangulate", 14, 15), ("t:gate", 14, 26), ("t:solve", 26, 27), ("t:append", 27, 15),
         ("total", 0, 15)]
acc = {k: [] for k, _, _ in names}
for i in range(2, n):
    eng.step(fr[i:i + 1])
    torch.cuda.synchronize()
    lib.vo_pnp_prof_read(buf)
    t = np.array(buf[:32], dtype=np.int64)
    row = {k: (t[b] - t[a]) / 100.0 for k, a, b in names}
    for k in row:
        acc[k].append(row[k])
    if i < 8 or i % 10 == 0:
        print(f"step {i}: " + " | ".join(f"{k} {v:6.1f}" for k, v in row.items()) +
              f" | hyps {t[20]} niters {t[21]} best {t[22]} | nL {int(eng.t['nL'][0])} nC {int(eng.t['nC'][0])}",
              flush=True)
print("median us: " + " | ".join(f"{k} {np.median(v[5:]):6.1f}" for k, v in acc.items()), flush=True)
