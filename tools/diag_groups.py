"""Bootstrap of the same chains as one engine vs G engines on G streams (not collected).

    python tests/diag_groups.py [B] [G]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from monocular_visual_odometry_va4mr_amd import options as Op  # noqa: E402
from monocular_visual_odometry_va4mr_amd.engine import Engine  # noqa: E402
from monocular_visual_odometry_va4mr_amd.synth import Renderer  # noqa: E402


def run(frames, K, opts, G, dev):
    B = frames.shape[1]
    bounds = [(g * B) // G for g in range(G + 1)]
    engs = [Engine(K, opts, frames.shape[-1], frames.shape[-2], batch=bounds[g + 1] - bounds[g], device=dev,
                   fcap=64) for g in range(G)]
    streams = [torch.cuda.Stream(dev) if G > 1 else torch.cuda.current_stream(dev) for _ in range(G)]
    torch.cuda.synchronize()
    for g, e in enumerate(engs):
        with torch.cuda.stream(streams[g]):
            e.bootstrap(frames[0, bounds[g]:bounds[g + 1]], frames[1, bounds[g]:bounds[g + 1]])
    torch.cuda.synchronize()
    st = np.concatenate([e.statuses() for e in engs])
    cnt = np.concatenate([e._boot_debug["cnt"].cpu().numpy() for e in engs])
    n0 = np.concatenate([e._boot_debug["n0"].cpu().numpy() for e in engs])
    n1 = np.concatenate([e._boot_debug["n1"].cpu().numpy() for e in engs])
    nL = np.concatenate([e.t["nL"].cpu().numpy() for e in engs])
    return st, cnt, n0, n1, nL


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    G = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    dev = torch.device("cuda", 0)
    opts, (b0, b1), _ = Op.get("kitti")
    rend = Renderer("kitti", seed=1, device=dev)
    gt = bench.StagePoses(bench.SEQ_LEN, rend.p)
    starts = [min((g * bench.SEQ_LEN) // B, bench.SEQ_LEN - 30) for g in range(B)]
    frames = bench.render_windows(rend, gt, starts, b1 - b0, 0, dev)
    torch.cuda.synchronize()
    a = run(frames, rend.K, opts, 1, dev)
    for rep in range(2):
        b = run(frames, rend.K, opts, G, dev)
        names = ["status", "cnt", "n0", "n1", "nL"]
        for n, x, y in zip(names, a, b):
            d = np.nonzero(x != y)[0]
            if len(d):
                print(f"rep {rep}: {n} differs at chains {d[:10].tolist()}: G1 {x[d[:10]].tolist()} G{G} {y[d[:10]].tolist()}")
    print("G1 statuses", np.unique(a[0], return_counts=True))


if __name__ == "__main__":
    main()
