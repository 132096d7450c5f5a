"""Single-chain leg of bench.py alone (drop-in class mode: one chain, host sync per frame),
eager and hipGraph, for kernel traces: python tools/single_prof.py [n_frames]."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from monocular_visual_odometry_va4mr_amd import options as Op  # noqa: E402
from monocular_visual_odometry_va4mr_amd.synth import Renderer  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
dev = torch.device("cuda")
opts, (b0, b1), _ = Op.get("kitti")
gap = b1 - b0
rend = Renderer("kitti", seed=1, device=dev)
gt = bench.StagePoses(n + gap + 8, rend.p)
sample = bench.render_windows(rend, gt, [0], gap, n - 2, dev)[:, 0]
pos, st, lat, lat_g, same = bench.gpu_chain_positions(rend.K, opts, sample, dev)
print(json.dumps({"frames_per_s": round(1 / lat, 1), "graph_frames_per_s": round(1 / lat_g, 1),
                  "ms": round(lat * 1e3, 4), "graph_ms": round(lat_g * 1e3, 4), "identical": same,
                  "status": int(st)}), flush=True)
