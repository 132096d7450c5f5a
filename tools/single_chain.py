#!/usr/bin/env python3
"""One chain through the drop-in class on KITTI-size frames (for rocprofv3 of the B=1 step).
usage: python tools/single_chain.py [n_frames] [graph 0/1]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from monocular_visual_odometry_va4mr_amd import options as Op  # noqa: E402
from monocular_visual_odometry_va4mr_amd.synth import Renderer, poses  # noqa: E402
from monocular_visual_odometry_va4mr_amd.VisualOdometryPipeLine import VisualOdometryPipeLine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 60
use_graph = bool(int(sys.argv[2])) if len(sys.argv) > 2 else True
rend = Renderer("kitti", seed=1, device="cuda")
Rs, cs = poses(n, rend.p)
fr = rend.render_batch(list(range(n)), Rs, cs)
opts, boot, _ = Op.get("kitti")
vo = VisualOdometryPipeLine(rend.K, opts, max_frames=n + 8, use_graph=use_graph)
vo.initialization(fr[boot[0]], fr[boot[1]])
torch.cuda.synchronize()
lat = []
for i in range(boot[1] + 1, n):
    t0 = time.perf_counter()
    vo.continuous_operation(fr[i])
    torch.cuda.synchronize()
    lat.append(time.perf_counter() - t0)
print(f"median {np.median(lat[5:]) * 1e3:.3f} ms/frame, {1.0 / np.median(lat[5:]):.1f} frames/s")
