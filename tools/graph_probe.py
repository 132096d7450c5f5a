#!/usr/bin/env python3
"""One KITTI chain, per-frame latency (step + status word + one host sync, as the drop-in class)
for the eager step and the captured step: frames read in place through the graph's frame slot,
or copied into the graph's buffer first.  Also the host-side time of each call (before the
sync).  usage: python tools/graph_probe.py [n_frames]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from monocular_visual_odometry_va4mr_amd import options as Op  # noqa: E402
from monocular_visual_odometry_va4mr_amd.engine import Engine  # noqa: E402
from monocular_visual_odometry_va4mr_amd.synth import Renderer, poses  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 120
rend = Renderer("kitti", seed=1, device="cuda")
Rs, cs = poses(n, rend.p)
fr = rend.render_batch(list(range(n)), Rs, cs)
opts, boot, _ = Op.get("kitti")


def chain(mode):
    eng = Engine(rend.K, opts, rend.W, rend.H, batch=1, ncap=16384, pcap=16384, fcap=n + 8)
    eng.bootstrap(fr[boot[0]:boot[0] + 1], fr[boot[1]:boot[1] + 1])
    if mode != "eager":
        eng.capture_step()
    torch.cuda.synchronize()
    lat, host = [], []
    for i in range(boot[1] + 1, n):
        f = fr[i:i + 1]
        t0 = time.perf_counter()
        if mode == "eager":
            eng.step(f)
        elif mode == "graph_slot":
            eng.step_graph(f)
        else:
            eng._graphs["buf"].copy_(f)
            eng.replay_step()
        t1 = time.perf_counter()
        eng.status_word(in_graph=mode != "eager")
        lat.append(time.perf_counter() - t0)
        host.append(t1 - t0)
    t = eng.t["pose_t"][0, :int(eng.t["nF"][0])].cpu().numpy()
    return np.median(lat[10:]) * 1e3, np.median(host[10:]) * 1e3, t


res = {}
for rep in range(2):
    for mode in ("eager", "graph_slot", "graph_copy"):
        ms, hms, t = chain(mode)
        res.setdefault(mode, []).append((round(ms, 4), round(hms, 4)))
        res.setdefault("t_" + mode, t)
same = all(np.array_equal(res["t_eager"], res["t_" + m]) for m in ("graph_slot", "graph_copy"))
print({m: res[m] for m in ("eager", "graph_slot", "graph_copy")}, "identical", same)
