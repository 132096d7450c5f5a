"""Why do chains of the synthetic KITTI-length sequence die?  (GPU box)

Runs the run_sequence shard plan (16 shards of the 4541-frame C2 sequence by default) as
the B chains of one Engine, recording per step and chain: landmarks N, candidates P,
PnP inliers and status.  For every chain that fails it prints the frame index, the status
and the counts over the preceding steps.
Usage: python tools/shard_diag.py [--frames 4541] [--shards 16] [--seed 1] [--preset kitti]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from monocular_visual_odometry_va4mr_amd import options as Op  # noqa: E402
from monocular_visual_odometry_va4mr_amd import shards as Sh  # noqa: E402
from monocular_visual_odometry_va4mr_amd.engine import Engine  # noqa: E402
from monocular_visual_odometry_va4mr_amd.synth import Renderer, poses  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=4541)
    ap.add_argument("--shards", type=int, default=16)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--preset", default="kitti")
    ap.add_argument("--out", default="gpurun_out/shard_diag.npz")
    a = ap.parse_args()
    dev = torch.device("cuda")
    opts, (b0, b1), _ = Op.get(a.preset)
    plan = Sh.plan_shards(a.frames, a.shards, b1 - b0, 30)
    B = len(plan)
    rend = Renderer(a.preset, seed=a.seed, device=dev)
    Rs, cs = poses(a.frames, rend.p)
    max_f = max(s.end - s.boot1 + 1 for s in plan)
    eng = Engine(rend.K, opts, rend.W, rend.H, batch=B, device=dev, fcap=max_f + 8)

    def frames_at(ids):
        ids = [min(int(i), a.frames - 1) for i in ids]
        return rend.render_batch(ids, Rs[ids], cs[ids])

    t0 = time.time()
    eng.bootstrap(frames_at([s.start for s in plan]), frames_at([s.boot1 for s in plan]))
    T = eng.t
    n_steps = max(s.n_steps for s in plan)
    hist = np.zeros((n_steps + 1, B, 4), np.int64)
    hist[0] = np.stack([T["nL"].cpu().numpy(), T["nC"].cpu().numpy(), T["nInl"].cpu().numpy(),
                        T["status"].cpu().numpy()], 1)
    for j in range(n_steps):
        eng.step(frames_at([min(s.boot1 + 1 + j, s.end - 1) for s in plan]))
        hist[j + 1] = np.stack([T["nL"].cpu().numpy(), T["nC"].cpu().numpy(), T["nInl"].cpu().numpy(),
                                T["status"].cpu().numpy()], 1)
        if j % 50 == 0:
            print(f"step {j}/{n_steps} alive {(hist[j + 1, :, 3] == 0).sum()}/{B} {time.time() - t0:.0f}s", flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    np.savez_compressed(a.out, hist=hist, starts=[s.start for s in plan], ends=[s.end for s in plan])
    for b, s in enumerate(plan):
        st = hist[:, b, 3]
        bad = np.nonzero(st != 0)[0]
        real_steps = s.n_steps
        if len(bad) == 0:
            print(f"shard {b} [{s.start},{s.end}) ok  N min {hist[:real_steps + 1, b, 0].min()} "
                  f"P min {hist[:real_steps + 1, b, 1].min()}")
            continue
        j = bad[0]
        frame = s.boot1 + j
        within = j <= real_steps
        print(f"shard {b} [{s.start},{s.end}) FAILED status {st[j]} at step {j} (frame {frame}, "
              f"{'inside' if within else 'after'} the shard)")
        lo = max(0, j - 12)
        for q in range(lo, j + 1):
            print(f"    step {q:4d} frame {s.boot1 + q:5d}: N {hist[q, b, 0]:5d} P {hist[q, b, 1]:5d} "
                  f"inl {hist[q, b, 2]:5d} st {hist[q, b, 3]}")


if __name__ == "__main__":
    main()
