"""Trajectory I/O and evaluation.

The reference reads ground truth for the plots only: KITTI `poses/00.txt` rows of a
row-major 3x4 [R|t] (utils.py:19-20, columns [-9] and [-1] = t_x, t_z) and the parking
`poses.txt` (utils.py:46-47).  It logs the estimated camera position
transforms[k][1] (main.py:121,172) and defines no error metric; here:

* read/write KITTI-format pose files (12 floats per line),
* absolute trajectory error (Umeyama Sim(3) RMSE, ate.py) and relative pose error over a
  frame gap (translation after a Sim(3) scale alignment, rotation in degrees),
* a report for sharded runs: per-shard ATE and the stitched trajectory's ATE.
"""
from __future__ import annotations

import numpy as np

from .ate import ate, umeyama


def read_kitti_poses(path: str) -> np.ndarray:
    """[n, 3, 4] camera-to-world poses from a KITTI-format text file."""
    a = np.loadtxt(path, dtype=np.float64, ndmin=2)
    if a.shape[1] != 12:
        raise ValueError(f"{path}: expected 12 values per line, got {a.shape[1]}")
    return a.reshape(-1, 3, 4)


def write_kitti_poses(path: str, transforms) -> None:
    """Write (R_CW, t_CW) pairs (the reference's ``transforms`` list) as KITTI rows."""
    rows = []
    for R, t in transforms:
        P = np.hstack([np.asarray(R, np.float64).reshape(3, 3), np.asarray(t, np.float64).reshape(3, 1)])
        rows.append(P.reshape(-1))
    np.savetxt(path, np.array(rows), fmt="%.12e")


def poses_from_transforms(transforms) -> np.ndarray:
    return np.stack([np.hstack([np.asarray(R, np.float64).reshape(3, 3),
                                np.asarray(t, np.float64).reshape(3, 1)]) for R, t in transforms])


def rpe(est: np.ndarray, ref: np.ndarray, delta: int = 1):
    """Relative pose error over `delta` frames between camera-to-world pose arrays [n,3,4].

    The estimate is first scaled by the Sim(3) scale that best aligns its positions to the
    reference (monocular VO has no metric scale).  Returns (translation RMSE, rotation
    RMSE in degrees)."""
    est = np.asarray(est, np.float64)
    ref = np.asarray(ref, np.float64)
    n = min(len(est), len(ref))
    if n <= delta:
        return 0.0, 0.0
    s, _, _ = umeyama(est[:n, :, 3], ref[:n, :, 3], True)
    te, re = [], []
    for i in range(n - delta):
        Re0, te0 = est[i, :, :3], est[i, :, 3] * s
        Re1, te1 = est[i + delta, :, :3], est[i + delta, :, 3] * s
        Rr0, tr0 = ref[i, :, :3], ref[i, :, 3]
        Rr1, tr1 = ref[i + delta, :, :3], ref[i + delta, :, 3]
        # relative motion in the first camera's frame
        dRe, dte = Re0.T @ Re1, Re0.T @ (te1 - te0)
        dRr, dtr = Rr0.T @ Rr1, Rr0.T @ (tr1 - tr0)
        E = dRr.T @ dRe
        te.append(np.linalg.norm(dte - dtr))
        c = np.clip((np.trace(E) - 1.0) * 0.5, -1.0, 1.0)
        re.append(np.degrees(np.arccos(c)))
    return float(np.sqrt(np.mean(np.square(te)))), float(np.sqrt(np.mean(np.square(re))))


def shard_report(shards, centres, gt_positions, stitched=None, reference=None) -> dict:
    """ATE of every shard against ground truth over its own frames (and, when ``reference``
    maps shard index -> the reference CPU path's positions on the same shard boundaries,
    against those: SURVEY.md §8e's parity definition), and of the stitched trajectory over
    the frames it covers.  A stitched result with coverage breaks is evaluated per segment
    (each segment Sim(3)-aligned on its own); the breaks are listed."""
    gt = np.asarray(gt_positions, np.float64)
    per = []
    for s, c in zip(shards, centres):
        fr = np.array([s.start] + list(range(s.boot1, s.end)))[:len(c)]
        if len(fr) >= 3:
            rmse, rel = ate(np.asarray(c)[:len(fr)], gt[fr])
            rec = {"shard": s.index, "frames": int(len(fr)), "ate_rmse": rmse, "ate_rel": rel}
            if reference is not None and s.index in reference:
                r = np.asarray(reference[s.index], np.float64)
                m = min(len(r), len(c))
                rec["ref_frames"] = int(m)
                rec["identical_to_ref"] = bool(len(r) == len(c) and np.array_equal(np.asarray(c), r))
                if m >= 3:
                    rr, rl = ate(np.asarray(c)[:m], r[:m])
                    rec["ate_vs_ref_rmse"], rec["ate_vs_ref_rel"] = rr, rl
            per.append(rec)
    out = {"shards": per}
    if stitched is not None:
        pos = stitched.positions
        n = min(len(pos), len(gt))
        segs = []
        for k in range(len(stitched.segments)):
            keep = stitched.segment[:n] == k
            if keep.sum() >= 3:
                rmse, rel = ate(pos[:n][keep], gt[:n][keep])
                segs.append({"shards": list(stitched.segments[k]), "frames": int(keep.sum()),
                             "ate_rmse": rmse, "ate_rel": rel})
        covered = int((stitched.segment[:n] >= 0).sum())
        out["stitched"] = {"frames": covered, "segments": segs,
                           "coverage_breaks": [list(b) for b in stitched.breaks]}
        if len(segs) == 1:
            out["stitched"]["ate_rmse"] = segs[0]["ate_rmse"]
            out["stitched"]["ate_rel"] = segs[0]["ate_rel"]
    return out
