#!/usr/bin/env python3
"""Host-side cost of one drop-in step (one KITTI chain, eager): per frame, the time from the call
to the first stage launch (Python before vo_pyr_build), the launch sequence, and the wait in
status_word; medians over the run.  usage: python tools/host_gap.py [n_frames]"""
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import bench  # noqa: E402
from monocular_visual_odometry_va4mr_amd import options as Op  # noqa: E402
from monocular_visual_odometry_va4mr_amd.engine import Engine  # noqa: E402
from monocular_visual_odometry_va4mr_amd.synth import Renderer  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 120
dev = torch.device("cuda")
opts, (b0, b1), _ = Op.get("kitti")
gap = b1 - b0
rend = Renderer("kitti", seed=1, device=dev)
gt = bench.StagePoses(n + gap + 8, rend.p)
fr = bench.render_windows(rend, gt, [0], gap, n - 2, dev)[:, 0]
eng = Engine(rend.K, opts, fr.shape[-1], fr.shape[-2], batch=1, device=dev, ncap=16384, pcap=16384, fcap=n + 8)
eng.bootstrap(fr[0:1], fr[1:2])
torch.cuda.synchronize()
marks_t = {}


def marks(i, end, strm):
    marks_t[(i, end)] = time.perf_counter()


rows = []
for i in range(2, n):
    marks_t.clear()
    t0 = time.perf_counter()
    eng.step(fr[i:i + 1], marks=marks)
    t1 = time.perf_counter()
    eng.status_word()
    t2 = time.perf_counter()
    rows.append((marks_t[(0, False)] - t0, t1 - marks_t[(0, False)], t2 - t1, t2 - t0))
r = np.array(rows[10:]) * 1e6
print("median us: pre-launch %.1f | launches %.1f | wait %.1f | frame %.1f" % tuple(np.median(r, axis=0)))
# the same frames without marks (the marks add host time)
lat = []
eng2 = Engine(rend.K, opts, fr.shape[-1], fr.shape[-2], batch=1, device=dev, ncap=16384, pcap=16384, fcap=n + 8)
eng2.bootstrap(fr[0:1], fr[1:2])
torch.cuda.synchronize()
for i in range(2, n):
    t0 = time.perf_counter()
    eng2.step(fr[i:i + 1])
    t1 = time.perf_counter()
    eng2.status_word()
    lat.append((t1 - t0, time.perf_counter() - t0))
r = np.array(lat[10:]) * 1e6
print("no marks, median us: step() host %.1f | frame %.1f" % tuple(np.median(r, axis=0)))
# the same frames replayed from the step hipGraph (step_graph: copy into the bound buffer, replay)
eng3 = Engine(rend.K, opts, fr.shape[-1], fr.shape[-2], batch=1, device=dev, ncap=16384, pcap=16384, fcap=n + 8)
eng3.bootstrap(fr[0:1], fr[1:2])
eng3.capture_step()
torch.cuda.synchronize()
lat = []
for i in range(2, n):
    t0 = time.perf_counter()
    eng3.step_graph(fr[i:i + 1])
    t1 = time.perf_counter()
    eng3.status_word(in_graph=True)
    lat.append((t1 - t0, time.perf_counter() - t0))
r = np.array(lat[10:]) * 1e6
print("graph, median us: step_graph() host %.1f | frame %.1f" % tuple(np.median(r, axis=0)))
# replay without the input copy (same frame buffer every time: timing only)
lat = []
for i in range(2, n):
    t0 = time.perf_counter()
    eng3.replay_step()
    t1 = time.perf_counter()
    eng3.status_word(in_graph=True)
    lat.append((t1 - t0, time.perf_counter() - t0))
r = np.array(lat[10:]) * 1e6
print("graph without the copy, median us: replay host %.1f | frame %.1f" % tuple(np.median(r, axis=0)))
