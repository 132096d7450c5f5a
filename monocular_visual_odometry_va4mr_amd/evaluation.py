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


def stitched_vs_one_chain(stitched, one_chain_t, boot1: int) -> dict | None:
    """The stitched multi-shard trajectory against the reference class run as ONE chain over
    the whole sequence (tests/golden/kitti_seq00.npz: t_CW of frames boot1, boot1 + 1, ...;
    SURVEY.md §8e's informational figure): Umeyama Sim(3) ATE over the frames both cover, in
    the stitched segment that covers most of them, relative to the one chain's path length.
    The monocular chain drifts in scale and is chaotic, so this measures how far
    two valid trajectories of the same frames are apart, not an error of either."""
    if stitched is None:
        return None
    ref = np.asarray(one_chain_t, np.float64)
    pos, seg = stitched.positions, stitched.segment
    frames = np.arange(boot1, boot1 + len(ref))
    frames = frames[frames < len(pos)]
    segs = seg[frames]
    ids, counts = np.unique(segs[segs >= 0], return_counts=True)
    if len(ids) == 0:
        return None
    keep = frames[segs == ids[np.argmax(counts)]]
    if len(keep) < 3:
        return None
    rmse, rel = ate(pos[keep], ref[keep - boot1])
    return {"frames": int(len(keep)), "ate_rmse": rmse, "ate_rel": rel}


def load_shard_cut(path: str, n_shards: int) -> dict | None:
    """One cut of a shard fixture (tests/golden/kitti_seq00_shards*.npz, written by
    make_long_golden.py from the reference class's own runs): per shard its (start, boot1,
    end) bounds and, per pose from the bootstrap pose on, t_CW and (num_pts, landmarks,
    candidates), plus the reference's error string ("" when it ran to the shard's end)."""
    import os
    if not os.path.exists(path):
        return None
    g = np.load(path, allow_pickle=False)
    key = f"s{n_shards}"
    if f"{key}_t" not in g.files:
        return None
    return {"bounds": g[f"{key}_bounds"], "t": g[f"{key}_t"], "counts": g[f"{key}_counts"],
            "off": g[f"{key}_off"], "error": g[f"{key}_error"]}


def chains_vs_shard_cut(cut: dict, starts, gap: int, pose_t, num_pts, nF, nL, nC, status, max_diffs: int = 16) -> dict:
    """Compare batched chains with the reference runs of a shard cut.

    A chain whose bootstrap frames [s, s + gap] are those of a shard of the cut ran exactly that
    shard's frames (the bench's chain g takes frame s_g + gap + j - 1 at step j >= 2, as the
    shard does), so its poses must equal the reference's pose for pose.  Per such chain, over
    the poses both have: every t_CW (pose 0 is the identity at s), num_pts; when the reference
    covers every pose of the chain, also the final landmark / candidate counts; a chain that
    still tracks where the reference crashed counts as different.  Arrays are the engine's:
    pose_t [B, fcap, 3] f64, num_pts [B, fcap] i32, nF / nL / nC / status [B]."""
    pose_t, num_pts = np.asarray(pose_t), np.asarray(num_pts)
    nF, nL, nC, status = (np.asarray(a).reshape(-1) for a in (nF, nL, nC, status))
    by_start = {int(b[0]): k for k, b in enumerate(cut["bounds"]) if int(b[1]) - int(b[0]) == gap}
    off = cut["off"]
    compared = identical = full = 0
    diffs = []
    for g, s in enumerate(starts):
        k = by_start.get(int(s))
        if k is None:
            continue
        t = cut["t"][off[k]:off[k + 1]]                 # poses 1 .. of the shard
        cnt = cut["counts"][off[k]:off[k + 1]]
        err = str(cut["error"][k])
        n = int(nF[g])                                  # chain poses incl. the identity
        m = min(n - 1, len(t))
        compared += 1
        ok = n >= 2 and bool(np.all(pose_t[g, 0] == 0.0))
        first = None
        if ok:
            eq = np.all(pose_t[g, 1:1 + m] == t[:m], axis=1) & (num_pts[g, 1:1 + m] == cnt[:m, 0])
            if not eq.all():
                ok, first = False, int(np.argmin(eq)) + 1
        covered = m == n - 1
        if ok and covered:
            full += 1
            if err and len(t) == m:
                # the reference crashed at its next frame: the chain must have stopped there too
                ok = int(status[g]) != 0 or n - 1 == 0
            else:
                ok = int(nL[g]) == int(cnt[m - 1, 1]) and int(nC[g]) == int(cnt[m - 1, 2]) and int(status[g]) == 0
            first = None if ok else n - 1
        elif ok and err:                               # the reference crashed before this chain's end
            ok, first = False, m + 1
        identical += int(ok)
        if not ok and len(diffs) < max_diffs:
            diffs.append({"chain": int(g), "shard": int(k), "first_pose": first, "status": int(status[g])})
    return {"compared": compared, "identical": identical, "covering_every_pose": full, "differences": diffs}
