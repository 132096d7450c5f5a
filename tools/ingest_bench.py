#!/usr/bin/env python3
"""Decode throughput of libvo_ingest on KITTI-size PNGs (writes them to a temp dir first).
usage: python tools/ingest_bench.py [n_frames] [threads]"""
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from PIL import Image  # noqa: E402
from monocular_visual_odometry_va4mr_amd import ingest  # noqa: E402
from monocular_visual_odometry_va4mr_amd.synth import make_sequence  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
threads = int(sys.argv[2]) if len(sys.argv) > 2 else 16
fr, _, _, _ = make_sequence("kitti", 8, seed=1)
d = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
paths = []
for i in range(n):
    p = os.path.join(d, f"{i:06d}.png")
    Image.fromarray(fr[i % 8], mode="L").save(p)
    paths.append(p)
B = 32
batches = [paths[i:i + B] for i in range(0, n - B + 1, B)]
for dev in (["cuda"] if len(sys.argv) > 3 and sys.argv[3] == "gpu" else ["cpu"]):
    src = ingest.FrameSource(batches, 1241, 376, device=dev, threads=threads)
    t0 = time.perf_counter()
    m = 0
    for b in src:
        m += b.shape[0]
    dt = time.perf_counter() - t0
    src.close()
    print(f'{{"ingest_frames_per_s": {m / dt:.1f}, "threads": {threads}, "frames": {m}, "device": "{dev}"}}')
