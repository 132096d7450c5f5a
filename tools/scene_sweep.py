"""Synthetic-scene sweep (GPU box): which SceneParams give a KITTI-size sequence that the
reference orchestration tracks end to end?

Each variant of synth.SceneParams is one chain of a batched Engine (bit-identical to the
reference class on the oracle, tests/test_gpu_*), bootstrapped at frames [0, 2] and stepped
over the whole sequence.  Reports per variant the frame at which the chain dies (if it
does), the landmark count range and the scale drift (estimated / true distance travelled
over successive 500-frame windows).
Usage: python tools/scene_sweep.py [--frames 4541] [--seed 1]
"""
import argparse
import dataclasses
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from monocular_visual_odometry_va4mr_amd import options as Op  # noqa: E402
from monocular_visual_odometry_va4mr_amd.engine import Engine  # noqa: E402
from monocular_visual_odometry_va4mr_amd.synth import Renderer, SceneParams  # noqa: E402

VARIANTS2 = {
    "sp0.5nolod": {"speed": 0.5, "lod": False, "octaves": 7},
    "sp0.4nolod": {"speed": 0.4, "lod": False, "octaves": 7},
    "sp0.6nolod": {"speed": 0.6, "lod": False, "octaves": 7},
    "sp0.5nolod8": {"speed": 0.5, "lod": False, "octaves": 8},
    "sp0.5nolod6": {"speed": 0.5, "lod": False, "octaves": 6},
    "sp0.5nolodn1": {"speed": 0.5, "lod": False, "octaves": 7, "noise_sigma": 1.0},
}

VARIANTS = {
    "base": {},
    "speed0.5": {"speed": 0.5},
    "wall14": {"wall": 14.0, "ceiling": 10.0},
    "oct7": {"octaves": 7},
    "nolod": {"lod": False, "octaves": 7},
    "yaw2": {"yaw_amp_deg": 2.0},
    "contrast": {"contrast": 120.0, "noise_sigma": 1.0},
    "sp0.7w12": {"speed": 0.7, "wall": 12.0},
    "wl4": {"base_wavelength": 4.0, "octaves": 8},
    "sp0.5oct7": {"speed": 0.5, "octaves": 7},
    "sp0.5w14": {"speed": 0.5, "wall": 14.0, "ceiling": 10.0},
    "sp0.5nolod": {"speed": 0.5, "lod": False, "octaves": 7},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=4541)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--only", default="")
    ap.add_argument("--shards", type=int, default=0, help="run each VARIANTS2 entry as this many shards")
    a = ap.parse_args()
    if a.shards:
        return sweep_shards(a)
    names = [n for n in VARIANTS if not a.only or n in a.only.split(",")]
    fields = {f.name for f in dataclasses.fields(SceneParams)}
    dev = torch.device("cuda")
    rends = []
    for n in names:
        kw = {k: v for k, v in VARIANTS[n].items() if k in fields}
        if len(kw) != len(VARIANTS[n]):
            print(f"variant {n}: unknown SceneParams keys skipped {set(VARIANTS[n]) - fields}")
        rends.append(Renderer("kitti", seed=a.seed, device=dev, params=SceneParams(**kw)))
    B = len(rends)
    opts, (b0, b1), _ = Op.get("kitti")
    r0 = rends[0]
    eng = Engine(r0.K, opts, r0.W, r0.H, batch=B, device=dev, fcap=a.frames + 8)
    gts = [r.gt_poses(a.frames) for r in rends]

    def frames_at(i):
        return torch.stack([r.render(i, gts[k][0][i], gts[k][1][i]) for k, r in enumerate(rends)])

    t0 = time.time()
    eng.bootstrap(frames_at(b0), frames_at(b1))
    T = eng.t
    death = [-1] * B
    nmin = [1 << 30] * B
    for i in range(b1 + 1, a.frames):
        eng.step(frames_at(i))
        if i % 25 == 0 or i == a.frames - 1:
            st = T["status"].cpu().numpy()
            nl = T["nL"].cpu().numpy()
            for b in range(B):
                if st[b] != 0 and death[b] < 0:
                    death[b] = i
                elif st[b] == 0:
                    nmin[b] = min(nmin[b], int(nl[b]))
            if i % 500 == 0:
                print(f"frame {i} alive {(st == 0).sum()}/{B} {time.time() - t0:.0f}s", flush=True)
            if (st != 0).all():
                break
    nF = T["nF"].cpu().numpy()
    pt = T["pose_t"].cpu().numpy()
    out = {}
    for b, n in enumerate(names):
        c = pt[b, 1:nF[b]]                           # t_CW of frames b1, b1+1, ...
        g = gts[b][1][b1:b1 + len(c)]
        drift = []
        for w0 in range(0, len(c) - 1, 500):
            w1 = min(len(c) - 1, w0 + 500)
            est = np.linalg.norm(np.diff(c[w0:w1 + 1], axis=0), axis=1).sum()
            tru = np.linalg.norm(np.diff(g[w0:w1 + 1], axis=0), axis=1).sum()
            drift.append(round(float(est / max(tru, 1e-9)), 4))
        out[n] = {"death_frame": death[b], "frames_tracked": int(nF[b]) - 1, "min_landmarks": nmin[b],
                  "scale_per_500": drift}
        print(n, json.dumps(out[n]), flush=True)


def sweep_shards(a):
    """Every VARIANTS2 scene cut into a.shards shards (shards.plan_shards, 30-frame overlap),
    all shards of all variants as the chains of one Engine; reports failed shards."""
    from monocular_visual_odometry_va4mr_amd import shards as Sh
    dev = torch.device("cuda")
    opts, (b0, b1), _ = Op.get("kitti")
    plan = Sh.plan_shards(a.frames, a.shards, b1 - b0, 30)
    names = list(VARIANTS2)
    rends = [Renderer("kitti", seed=a.seed, device=dev, params=SceneParams(**VARIANTS2[n])) for n in names]
    gts = [r.gt_poses(a.frames) for r in rends]
    chains = [(v, s) for v in range(len(names)) for s in plan]
    B = len(chains)
    r0 = rends[0]
    max_f = max(s.end - s.boot1 + 1 for s in plan)
    eng = Engine(r0.K, opts, r0.W, r0.H, batch=B, device=dev, fcap=max_f + 8)

    def frames_at(ids):
        out = []
        for (v, _), i in zip(chains, ids):
            i = min(int(i), a.frames - 1)
            out.append(rends[v].render(i, gts[v][0][i], gts[v][1][i]))
        return torch.stack(out)

    t0 = time.time()
    eng.bootstrap(frames_at([s.start for _, s in chains]), frames_at([s.boot1 for _, s in chains]))
    T = eng.t
    n_steps = max(s.n_steps for s in plan)
    dead_at = np.full(B, -1)
    for j in range(n_steps):
        eng.step(frames_at([s.boot1 + 1 + j if j < s.n_steps else s.end - 1 for _, s in chains]))
        st = T["status"].cpu().numpy()
        for c in range(B):
            if st[c] != 0 and dead_at[c] < 0 and j < chains[c][1].n_steps:
                dead_at[c] = chains[c][1].boot1 + 1 + j
        if j % 50 == 0:
            print(f"step {j}/{n_steps} {time.time() - t0:.0f}s", flush=True)
    for v, n in enumerate(names):
        dead = [(s.index, int(dead_at[c])) for c, (vv, s) in enumerate(chains) if vv == v and dead_at[c] >= 0]
        print(n, json.dumps({"shards": len(plan), "failed": dead}), flush=True)


if __name__ == "__main__":
    main()
