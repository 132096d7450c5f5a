"""The CPU oracle restatement reproduces the reference class bit for bit.

tests/golden/*.npz were produced by the reference's own VisualOdometryPipeLine
(/root/reference/VisualOdometryPipeLine.py) driven by oracle/cv2_oracle.py
(tests/golden/make_golden.py).  Here the restatement oracle/vo_pipeline_oracle.py is
run on the same (re-rendered, digest-checked) frames and must match exactly.
"""
import numpy as np
import pytest

from conftest import golden_frames, load_golden


def _run_restatement(g, n_steps=None):
    from oracle import vo_pipeline_oracle as V
    from monocular_visual_odometry_va4mr_amd import options as O
    fr = golden_frames(g)
    opts, boot, _ = O.get(str(g["preset"]))
    s = V.new_state(g["K"], opts)
    V.initialize(s, fr[boot[0]], fr[boot[1]])
    rows = [(s.transforms[-1], s.num_pts[-1], len(s.lm), s.cand.shape[0])]
    snaps = {boot[1]: (s.lm.copy(), s.kp.copy(), s.cand.copy(), s.cand_first.copy(), s.cand_tau.copy())}
    frames = list(g["frame"][1:])
    if n_steps is not None:
        frames = frames[:n_steps]
    for i in frames:
        V.step(s, fr[i])
        rows.append((s.transforms[-1], s.num_pts[-1], len(s.lm), s.cand.shape[0]))
        snaps[int(i)] = (s.lm.copy(), s.kp.copy(), s.cand.copy(), s.cand_first.copy(), s.cand_tau.copy())
    return rows, snaps


@pytest.mark.parametrize("case,n_steps", [("kitti_c2", 40), ("parking_c1", 30), ("malaga_c3", None),
                                          ("malaga1024_c3", 12)])
def test_restatement_matches_reference(case, n_steps):
    g = load_golden(case)
    rows, snaps = _run_restatement(g, n_steps)
    for k, ((R, t), num, N, P) in enumerate(rows):
        assert np.array_equal(R, g["R"][k]), f"R differs at record {k}"
        assert np.array_equal(t, g["t"][k]), f"t differs at record {k}"
        assert num == g["num_pts"][k] and N == g["N"][k] and P == g["P"][k]
    for i, (lm, kp, c, cf, ct) in snaps.items():
        if f"lm_{i}" in g:
            assert np.array_equal(lm, g[f"lm_{i}"])
            assert np.array_equal(kp, g[f"kp_{i}"])
            assert np.array_equal(c, g[f"cand_{i}"])
            assert np.array_equal(cf, g[f"cand_first_{i}"])
            assert np.array_equal(ct, g[f"cand_tau_{i}"])


def test_golden_sanity():
    """The recorded reference runs are non-degenerate (landmarks tracked, poses moving)."""
    for case in ("parking_c1", "kitti_c2", "malaga_c3", "malaga1024_c3"):
        g = load_golden(case)
        assert str(g["error"]) == ""
        assert (g["N"] >= 8).all()
        z = g["t"][:, 2, 0]
        assert z[-1] > z[0] + 1.0


def test_wide_shard_fixtures_consistent_and_pinned():
    """The sequence job's shard fixtures (kitti_seq00_shards*.npz, make_long_golden.py --cuts):
    shard 0 of every cut bootstraps at frame 0 like the one-chain run, so its trajectory is
    a prefix of kitti_seq00.npz, and its bounds are shards.plan_shards' for its overlap (30, and
    the sequence job's 15); and the restatement reproduces a whole shard of the widest 15-frame
    cut (its last one) from frames re-rendered here and checked against the digests."""
    import os
    from conftest import GOLDEN
    full = load_golden("kitti_seq00")
    cuts = {}
    for name in ("kitti_seq00_shards", "kitti_seq00_shards_wide", "kitti_seq00_shards_o15"):
        if os.path.exists(os.path.join(GOLDEN, f"{name}.npz")):
            g = load_golden(name)
            for k in g:
                if k.endswith("_t"):
                    cuts[(int(k[1:-2]), int(g["overlap"]))] = g
    assert {(8, 30), (16, 30), (256, 30), (256, 15)}.issubset(cuts)
    from monocular_visual_odometry_va4mr_amd import shards as Sh
    for (S, O), g in cuts.items():
        t, off = g[f"s{S}_t"], g[f"s{S}_off"]
        assert len(off) == S + 1 and off[-1] == len(t)
        assert all(str(e) == "" for e in g[f"s{S}_error"])
        assert np.array_equal(g[f"s{S}_bounds"], [[s.start, s.boot1, s.end] for s in Sh.plan_shards(4541, S, 2, O)])
        assert np.array_equal(t[off[0]:off[1]], full["t"][:off[1] - off[0]]), f"cut {S}/{O}: shard 0 is not the chain's prefix"
    S = 256
    g = cuts[(S, 15)]
    start, boot1, end = (int(v) for v in g[f"s{S}_bounds"][-1])
    import hashlib
    import torch
    from oracle import vo_pipeline_oracle as V
    from monocular_visual_odometry_va4mr_amd import options as O
    from monocular_visual_odometry_va4mr_amd.synth import Renderer
    r = Renderer(str(full["preset"]), seed=int(full["seed"]))
    Rs, cs = r.gt_poses(int(full["n_frames"]))
    ids = [start] + list(range(boot1, end))
    with torch.no_grad():
        fr = r.render_batch(ids, Rs[ids], cs[ids]).numpy()
    for i, f in zip(ids, fr):
        assert np.array_equal(np.frombuffer(hashlib.sha1(f.tobytes()).digest(), np.uint8), full["digests"][i])
    opts, _, _ = O.get(str(full["preset"]))
    s = V.new_state(r.K, opts)
    V.initialize(s, fr[0], fr[1])
    got = [np.asarray(s.transforms[-1][1], np.float64).ravel()]
    for f in fr[2:]:
        V.step(s, f)
        got.append(np.asarray(s.transforms[-1][1], np.float64).ravel())
    off = g[f"s{S}_off"]
    assert np.array_equal(np.stack(got), g[f"s{S}_t"][off[-2]:off[-1]])
