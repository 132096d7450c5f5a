#!/usr/bin/env python3
"""Seed-to-seed spread of the monocular chain against the OpenCV-form and SVD-form gaps
(CPU only, build container).

For seeds 0..7 of C1 (Parking 640x480, 100 frames) and C2 (KITTI 1241x376, the first
--c2-frames frames), the oracle restatement (oracle/vo_pipeline_oracle.py -- bit-identical to
the reference class on the oracle primitives, tests/test_oracle_golden.py) runs one chain from
the preset's bootstrap pair in three forms:

  int     the parity oracle (integer-exact GFTT / LK sums): what the GPU reproduces bit for bit
  lk32    LK window sums accumulated in float, OpenCV's form (vo_o_set_fp32_mode(2))
  svd2    EPnP's 12x12 SVD in the round-2 serial order (vo_o_set_svd_form(1))

and every trajectory is scored against ground truth (camera centres of the renderer; Umeyama
Sim(3) RMSE / ground-truth path length) and against the `int` run of the same seed.
--c2-full additionally runs the whole 4541-frame seed-1 chain in the svd2 form (frames from
make_long_golden.py's memmap) and compares it with kitti_seq00.npz (stop frame, ATE).

    python tools/seed_spread.py [--procs 7] [--c2-frames 1000] [--c2-full]

Writes profiles/r4_seed_spread.json.
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
OUT = os.environ.get("VO_SEED_SPREAD_OUT", os.path.join(REPO, "profiles", "r4_seed_spread.json"))
FORMS = {"int": (0, 0), "lk32": (2, 0), "svd2": (0, 1)}


def _chain(preset, frames, fp32_mode, svd_form):
    from oracle import _olib as O
    from oracle import vo_pipeline_oracle as V
    from monocular_visual_odometry_va4mr_amd import options as Op
    from monocular_visual_odometry_va4mr_amd.synth import intrinsics
    opts, (b0, b1), _ = Op.get(preset)
    O.set_fp32_mode(fp32_mode)
    O.set_svd_form(svd_form)
    err = ""
    try:
        s = V.new_state(intrinsics(preset), opts)
        V.initialize(s, np.asarray(frames[b0]), np.asarray(frames[b1]))
        pos = [np.asarray(t, np.float64).ravel() for _, t in s.transforms]     # frames b0, b1
        for i in range(b1 + 1, len(frames)):
            try:
                V.step(s, np.asarray(frames[i]))
            except Exception as e:  # noqa: BLE001 -- the reference's ValueErrors end the chain
                err = f"{type(e).__name__}: {e} (frame {i})"
                break
            pos.append(np.asarray(s.transforms[-1][1], np.float64).ravel())
    finally:
        O.set_fp32_mode(0)
        O.set_svd_form(0)
    return np.stack(pos), err


def _job(args):
    preset, seed, n = args
    import torch
    torch.set_num_threads(1)
    from monocular_visual_odometry_va4mr_amd.synth import Renderer
    from monocular_visual_odometry_va4mr_amd import options as Op
    from monocular_visual_odometry_va4mr_amd.ate import ate
    t0 = time.time()
    r = Renderer(preset, seed=seed)
    Rs, cs = r.gt_poses(n)
    frames = np.concatenate([r.render_batch(list(range(a, min(n, a + 8))), Rs[a:a + 8], cs[a:a + 8]).numpy()
                             for a in range(0, n, 8)])
    t_render = time.time() - t0
    _, (b0, b1), _ = Op.get(preset)
    out = {"preset": preset, "seed": seed, "frames": n, "render_s": round(t_render, 1)}
    runs = {}
    for name, (fm, sf) in FORMS.items():
        pos, err = _chain(preset, frames, fm, sf)
        ids = np.array([b0] + list(range(b1, b1 + len(pos) - 1)))
        rmse, rel = ate(pos, cs[ids])
        runs[name] = pos
        out[name] = {"poses": int(len(pos)), "error": err, "ate_vs_gt_rel": float(rel), "ate_vs_gt_rmse": float(rmse)}
    for name in ("lk32", "svd2"):
        m = min(len(runs[name]), len(runs["int"]))
        same = len(runs[name]) == len(runs["int"]) and bool(np.array_equal(runs[name], runs["int"]))
        first = np.nonzero((runs[name][:m] != runs["int"][:m]).any(1))[0]
        out[name]["identical_to_int"] = same
        out[name]["first_diff_pose"] = int(first[0]) if len(first) else None
        out[name]["ate_vs_int_rel"] = float(ate(runs[name][:m], runs["int"][:m])[1]) if m >= 3 else None
    print(f"  {preset} seed {seed}: " + ", ".join(
        f"{k} {out[k]['poses']} poses ate/gt {out[k]['ate_vs_gt_rel']:.4f}" for k in FORMS), flush=True)
    return out


def _full_svd2():
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    import make_long_golden as MLG
    from monocular_visual_odometry_va4mr_amd.ate import ate
    from monocular_visual_odometry_va4mr_amd.synth import SIZES
    g = np.load(os.path.join(REPO, "tests", "golden", "kitti_seq00.npz"), allow_pickle=False)
    W, H = SIZES["kitti"]
    n = int(g["n_frames"])
    mm = np.memmap(MLG.MEMMAP, np.uint8, "r", shape=(n, H, W))
    pos, err = _chain("kitti", mm, 0, 1)
    ref = np.concatenate([np.zeros((1, 3)), g["t"]])
    m = min(len(pos), len(ref))
    first = np.nonzero((pos[:m] != ref[:m]).any(1))[0]
    return {"case": "C2 seed 1, whole 4541-frame chain, EPnP SVD in the round-2 serial form",
            "poses": int(len(pos)), "error": err, "reference_poses": int(len(ref)),
            "reference_error": str(g["error"]), "first_diff_pose": int(first[0]) if len(first) else None,
            "ate_vs_golden_rel": float(ate(pos[:m], ref[:m])[1])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=7)
    ap.add_argument("--c2-frames", type=int, default=1000)
    ap.add_argument("--seeds", default="0,1,2,3,4,5,6,7")
    ap.add_argument("--c2-full", action="store_true")
    a = ap.parse_args()
    seeds = [int(s) for s in a.seeds.split(",")]
    jobs = [("kitti", s, a.c2_frames) for s in seeds] + [("parking", s, 100) for s in seeds]
    t0 = time.time()
    with mp.get_context("fork").Pool(a.procs) as pool:
        res = pool.map(_job, jobs, chunksize=1)
    summary = {}
    for preset in ("parking", "kitti"):
        rs = [r for r in res if r["preset"] == preset]
        gt = np.array([r["int"]["ate_vs_gt_rel"] for r in rs])
        summary[preset] = {
            "seeds": len(rs),
            "int_ate_vs_gt_rel": {"mean": float(gt.mean()), "std": float(gt.std()), "min": float(gt.min()),
                                  "max": float(gt.max())},
            "lk32_minus_int_ate_vs_gt_rel": [r["lk32"]["ate_vs_gt_rel"] - r["int"]["ate_vs_gt_rel"] for r in rs],
            "lk32_ate_vs_int_rel": [r["lk32"]["ate_vs_int_rel"] for r in rs],
            "svd2_ate_vs_int_rel": [r["svd2"]["ate_vs_int_rel"] for r in rs],
        }
    out = {"tool": "tools/seed_spread.py", "c2_frames": a.c2_frames, "runs": res, "summary": summary,
           "wall_s": round(time.time() - t0, 1)}
    if a.c2_full:
        out["c2_full_svd2"] = _full_svd2()
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
