#!/usr/bin/env python3
"""Trajectory-level bound on the oracle's two deliberate departures from OpenCV's fp32
arithmetic (CPU only, build container).

The oracle -- and bit for bit the HIP path -- computes goodFeaturesToTrack's covariance /
lambda_min exactly in integers (OpenCV: fp32 Sobel, double box sums, fp32 lambda) and the
LK window sums exactly in int64 (OpenCV: fp32 accumulation).  oracle/vo_oracle_img.c also
restates OpenCV's fp32 forms (vo_o_set_fp32_mode: bit 0 GFTT, bit 1 LK).  This script runs the
reference class (/root/reference/VisualOdometryPipeLine.py, imported unchanged with the oracle
shim as ``cv2``, as make_golden.py does) with those fp32 forms switched on, over

  kitti_seq00     the whole 4541-frame C2 sequence as one chain (golden kitti_seq00.npz)
  parking_c1      100 frames (golden parking_c1.npz)
  malaga1024_c3   40 frames (golden malaga1024_c3.npz)

for modes 1 (GFTT fp32), 2 (LK fp32 sums) and 3 (both), and stores every trajectory as a
fixture (tests/golden/opencv_fp32_trajectories.npz).  tests/test_opencv_deviation.py reports
the ATE (Umeyama Sim(3) RMSE relative to the path length) of each against the
integer-mode golden -- the trajectory the GPU reproduces bit for bit -- next to north_star's
1 % tolerance.  Usage: python tools/opencv_trajectory_bound.py [--procs 6] [--cases ...]
[--summary-only]; the ATE table (against the integer golden) goes to
profiles/r3_opencv_fp32_trajectory.json.
"""
from __future__ import annotations

import argparse
import multiprocessing as mp
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
OUT = os.path.join(REPO, "tests", "golden", "opencv_fp32_trajectories.npz")
LONG_MEMMAP = "/tmp/vo_long_golden_frames.u8"

CASES = {
    # name: (preset, seed, n_frames)
    "kitti_seq00": ("kitti", 1, 4541),
    "parking_c1": ("parking", 0, 100),
    "malaga1024_c3": ("malaga1024", 2, 40),
}
MODES = (1, 2, 3)


def _frames(case):
    preset, seed, n = CASES[case]
    if case == "kitti_seq00":
        sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
        import make_long_golden as MLG
        from monocular_visual_odometry_va4mr_amd.synth import SIZES
        W, H = SIZES[preset]
        shape = (n, H, W)
        if not os.path.exists(MLG.MEMMAP) or os.path.getsize(MLG.MEMMAP) != n * H * W:
            np.memmap(MLG.MEMMAP, np.uint8, "w+", shape=shape).flush()
            MLG._render_chunk((0, n, shape))
        return np.memmap(MLG.MEMMAP, np.uint8, "r", shape=shape)
    from monocular_visual_odometry_va4mr_amd.synth import make_sequence
    return make_sequence(preset, n, seed=seed)[0]


def _run(args):
    case, mode = args
    import oracle.cv2_oracle as cv2_oracle
    from oracle import _olib as O
    sys.modules["cv2"] = cv2_oracle
    sys.path.insert(0, "/root/reference")
    import VisualOdometryPipeLine as ref  # the reference module, unmodified
    from monocular_visual_odometry_va4mr_amd import options as Op
    from monocular_visual_odometry_va4mr_amd.synth import intrinsics
    O.set_fp32_mode(mode)
    preset, seed, n = CASES[case]
    fr = _frames(case)
    opts, (b0, b1), _ = Op.get(preset)
    vo = ref.VisualOdometryPipeLine(intrinsics(preset), opts)
    t0 = time.time()
    vo.initialization(np.array(fr[b0]), np.array(fr[b1]))
    ts = [np.asarray(vo.transforms[-1][1], np.float64).ravel().copy()]
    npts = [int(vo.num_pts[-1])]
    err = ""
    for i in range(b1 + 1, n):
        try:
            vo.continuous_operation(np.array(fr[i]))
        except Exception as e:  # the reference raises here; record where
            err = f"{type(e).__name__}: {e} (frame {i})"
            break
        ts.append(np.asarray(vo.transforms[-1][1], np.float64).ravel().copy())
        npts.append(int(vo.num_pts[-1]))
    print(f"  {case} mode {mode}: {len(ts)} poses in {time.time() - t0:.0f}s {err}", flush=True)
    return case, mode, np.stack(ts), np.array(npts, np.int32), err


def summary(path=os.path.join(REPO, "profiles", "r3_opencv_fp32_trajectory.json")):
    """ATE of every fp32-mode trajectory against the integer golden (over the poses both runs
    have)."""
    import json
    from monocular_visual_odometry_va4mr_amd.ate import ate
    fx = np.load(OUT, allow_pickle=False)
    rep = {"tool": "tools/opencv_trajectory_bound.py", "fixture": "tests/golden/opencv_fp32_trajectories.npz",
           "ate": "Umeyama Sim(3) RMSE / path length of the integer-mode trajectory, over the poses both runs have",
           "north_star_tolerance": 0.01, "cases": {}}
    for case in CASES:
        g = np.load(os.path.join(REPO, "tests", "golden", f"{case}.npz"), allow_pickle=False)
        ref = g["t"].reshape(len(g["t"]), 3)
        c = {"frames": int(len(ref)), "error": str(g["error"])}
        for m, name in ((1, "gftt_fp32"), (2, "lk_fp32_sums"), (3, "both")):
            t = fx[f"{case}_m{m}_t"]
            k = min(len(t), len(ref))
            c[name] = {"frames": int(len(t)), "error": str(fx[f"{case}_m{m}_error"]),
                       "identical_to_integer_golden": bool(len(t) == len(ref) and np.array_equal(t, ref)),
                       "ate_vs_integer": float(ate(t[:k], ref[:k])[1])}
        rep["cases"][case] = c
    with open(path, "w") as f:
        json.dump(rep, f, indent=1)
    print("wrote", path)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=6)
    ap.add_argument("--cases", nargs="*", default=list(CASES))
    ap.add_argument("--summary-only", action="store_true")
    a = ap.parse_args()
    if a.summary_only:
        summary()
        return
    for c in a.cases:           # render the long sequence once, before the workers fork
        if c == "kitti_seq00":
            _frames(c)
    jobs = [(c, m) for c in a.cases for m in MODES]
    jobs.sort(key=lambda j: -CASES[j[0]][2])          # longest first
    out = dict(np.load(OUT, allow_pickle=False)) if os.path.exists(OUT) else {}
    with mp.get_context("fork").Pool(min(a.procs, len(jobs))) as pool:
        for case, mode, t, npts, err in pool.imap_unordered(_run, jobs):
            out[f"{case}_m{mode}_t"] = t
            out[f"{case}_m{mode}_num_pts"] = npts
            out[f"{case}_m{mode}_error"] = np.asarray(err)
            np.savez_compressed(OUT, **out)             # keep what is done so far
    print("wrote", OUT)
    summary()


if __name__ == "__main__":
    main()
