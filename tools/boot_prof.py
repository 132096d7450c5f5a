"""bench.py's bootstrap of 768 chains (2 engines x 384, KITTI C2) alone, timed twice (first call
allocates the SIFT scale spaces), for kernel traces: python tools/boot_prof.py [chains]."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from monocular_visual_odometry_va4mr_amd import options as Op  # noqa: E402
from monocular_visual_odometry_va4mr_amd.engine import Engine  # noqa: E402
from monocular_visual_odometry_va4mr_amd.synth import Renderer  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 768
dev = torch.device("cuda")
opts, (b0, b1), _ = Op.get("kitti")
gap = b1 - b0
rend = Renderer("kitti", seed=1, device=dev)
gt = bench.StagePoses(bench.SEQ_LEN, rend.p)
starts = [min((g * bench.SEQ_LEN) // B, bench.SEQ_LEN - gap - 40) for g in range(B)]
frames = bench.render_windows(rend, gt, starts, gap, 0, dev)
G = int(os.environ.get("BOOT_GROUPS", "2"))
bounds = [(g * B) // G for g in range(G + 1)]
engines = [Engine(rend.K, opts, rend.W, rend.H, batch=bounds[g + 1] - bounds[g], device=dev, ncap=16384, pcap=16384,
                  fcap=64) for g in range(G)]
streams = [torch.cuda.Stream(dev) for _ in range(G)]
torch.cuda.synchronize()
t0 = time.perf_counter()
for g, e in enumerate(engines):
    with torch.cuda.stream(streams[g]):           # as bench.py: brings up the group's stream too
        e.reserve_bootstrap()
torch.cuda.synchronize()
print(f"workspace {time.perf_counter() - t0:.3f} s", flush=True)
for rep in range(3):
    t0 = time.perf_counter()
    for g, e in enumerate(engines):
        with torch.cuda.stream(streams[g]):
            e.bootstrap(frames[0, bounds[g]:bounds[g + 1]], frames[1, bounds[g]:bounds[g + 1]])
    torch.cuda.synchronize()
    print(f"bootstrap of {B} chains, call {rep}: {time.perf_counter() - t0:.3f} s", flush=True)
