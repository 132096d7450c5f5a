"""GPU bootstrap primitives (SIFT, BF kNN, E-RANSAC, recoverPose) and the full drop-in
pipeline vs the CPU oracle / reference-generated golden trajectories."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def test_bf_knn2_exact():
    from oracle import _olib as O
    from monocular_visual_odometry_va4mr_amd import cv2compat as G
    rng = np.random.default_rng(0)
    for nq, nt in [(300, 500), (129, 1), (70, 33), (1000, 2048)]:
        q = rng.integers(0, 256, (nq, 128)).astype(np.float32)
        t = rng.integers(0, 256, (nt, 128)).astype(np.float32)
        if nt > 10:
            t[5] = t[7]            # exact tie: the lower train index must win
            q[3] = t[5]
        m = G.BFMatcher().knnMatch(q, t, k=2)
        idx, dist = O.bf_knn2(q, t)
        for i in range(nq):
            assert len(m[i]) == (2 if nt >= 2 else 1)
            for j, dm in enumerate(m[i]):
                assert dm.trainIdx == idx[i, j] and np.float32(dm.distance) == dist[i, j]


def test_bf_knn2_i8_equals_bf16_at_c5_size(monkeypatch):
    """The int8 MFMA kernel (default) and the bf16 one (VO_BF_BF16=1) at BASELINE C5's full
    size, 2 x 8192 x 8192 with extreme (0/255-heavy) rows mixed in: identical indices and
    distances -- a size-independent property where the C oracle would take minutes."""
    from monocular_visual_odometry_va4mr_amd.features import bf_knn2_batch
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(5)
    q = torch.randint(0, 256, (2, 8192, 128), generator=g).float()
    t = torch.randint(0, 256, (2, 8192, 128), generator=g).float()
    q[:, :64] = 255.0 * (q[:, :64] > 127)
    t[:, :64] = 255.0 * (t[:, :64] < 128)
    t[:, 100] = t[:, 99]
    nq = torch.tensor([8192, 8000], dtype=torch.int32, device=dev)
    nt = torch.tensor([8192, 7777], dtype=torch.int32, device=dev)
    q, t = q.to(dev), t.to(dev)
    monkeypatch.delenv("VO_BF_BF16", raising=False)
    i8 = bf_knn2_batch(q, nq, t, nt)
    torch.cuda.synchronize()
    monkeypatch.setenv("VO_BF_BF16", "1")
    bf = bf_knn2_batch(q, nq, t, nt)
    torch.cuda.synchronize()
    assert torch.equal(i8[0], bf[0]) and torch.equal(i8[1], bf[1])


def test_bf_knn2_batch_exact():
    """Batched MFMA matcher vs the C restatement: ragged / empty problems, an exact tie, and
    0/255 descriptors whose distances^2 pass 2^22 (the exact float-order fixup path)."""
    from oracle import _olib as O
    from monocular_visual_odometry_va4mr_amd.features import bf_knn2_batch, matcher_scratch_bytes
    rng = np.random.default_rng(1)
    qcap, tcap = 700, 900
    sizes = [(700, 900), (1, 2), (0, 5), (333, 1), (650, 0), (129, 64), (300, 257)]
    B = len(sizes)
    q = np.zeros((B, qcap, 128), np.float32)
    t = np.zeros((B, tcap, 128), np.float32)
    for b, (nq, nt) in enumerate(sizes):
        if b == 6:      # 0/255 descriptors, mostly opposite: d2 = 65025 * hamming >= 2^22
            q[b, :nq] = 255 * (rng.random((nq, 128)) < 0.9)
            t[b, :nt] = 255 * (rng.random((nt, 128)) < 0.1)
        else:
            q[b, :nq] = rng.integers(0, 256, (nq, 128))
            t[b, :nt] = rng.integers(0, 256, (nt, 128))
        if nt > 10 and nq > 3:
            t[b, 7] = t[b, 5]          # exact tie: the lower train index must win
            q[b, 3] = t[b, 5]
    dev = torch.device("cuda")
    nq_d = torch.tensor([s[0] for s in sizes], dtype=torch.int32, device=dev)
    nt_d = torch.tensor([s[1] for s in sizes], dtype=torch.int32, device=dev)
    idx2, dist2 = bf_knn2_batch(torch.from_numpy(q).to(dev), nq_d, torch.from_numpy(t).to(dev), nt_d)
    idx2, dist2 = idx2.cpu().numpy(), dist2.cpu().numpy()
    big = 0
    for b, (nq, nt) in enumerate(sizes):
        if nq == 0:
            assert (idx2[b] == -1).all()
            continue
        if nt == 0:
            assert (idx2[b, :nq] == -1).all() and (dist2[b, :nq] == np.finfo(np.float32).max).all()
            continue
        ei, ed = O.bf_knn2(np.ascontiguousarray(q[b, :nq]), np.ascontiguousarray(t[b, :nt]))
        k = min(2, nt)
        assert np.array_equal(idx2[b, :nq, :k], ei[:, :k]), f"problem {b}"
        assert np.array_equal(dist2[b, :nq, :k], ed[:, :k]), f"problem {b}"
        if nt < 2:
            assert (idx2[b, :nq, 1] == -1).all()
        big += int((ed[:, 1] >= 2048.0).sum())
    assert big > 0          # the fixup path ran
    # the capacity plan (one item per block from the buffer sizes, VO_BF_PLAN=0) gives the same
    # result as the default device plan (splits from the real counts)
    import os
    os.environ["VO_BF_PLAN"] = "0"
    try:
        i4, d4 = bf_knn2_batch(torch.from_numpy(q).to(dev), nq_d, torch.from_numpy(t).to(dev), nt_d)
        torch.cuda.synchronize()
    finally:
        del os.environ["VO_BF_PLAN"]
    assert np.array_equal(i4.cpu().numpy(), idx2) and np.array_equal(d4.cpu().numpy(), dist2)
    # a caller-owned scratch buffer (what an Engine passes) gives the same result
    scr = torch.empty(matcher_scratch_bytes(B, qcap, tcap), dtype=torch.uint8, device=dev)
    i3, d3 = bf_knn2_batch(torch.from_numpy(q).to(dev), nq_d, torch.from_numpy(t).to(dev), nt_d, scratch=scr)
    assert np.array_equal(i3.cpu().numpy(), idx2) and np.array_equal(d3.cpu().numpy(), dist2)


@pytest.mark.parametrize("preset,seed", [("parking", 4), ("kitti", 1), ("malaga1024", 2), ("hd1080", 3)])
def test_sift_matches_oracle(preset, seed):
    """detectAndCompute (:226-227) bit for bit against the C restatement at every BASELINE
    image size: C1 640x480, C2 1241x376, C3 1024x768, C5 1920x1080 -- keypoint order,
    x, y, size, angle, response, octave and all 128 descriptor bins."""
    from oracle import _olib as O
    from monocular_visual_odometry_va4mr_amd import cv2compat as G
    from monocular_visual_odometry_va4mr_amd.synth import make_sequence
    fr, _, _, _ = make_sequence(preset, 1, seed=seed)
    kps, desc = G.SIFT_create().detectAndCompute(fr[0], None)
    ko, do = O.sift(fr[0])
    kg = np.array([[k.pt[0], k.pt[1], k.size, k.angle, k.response, k.octave] for k in kps], np.float32)
    assert len(kg) == len(ko) > 300
    assert np.array_equal(kg, ko)
    assert np.array_equal(desc, do)


def test_essential_and_recover_pose():
    from oracle import _olib as O
    from monocular_visual_odometry_va4mr_amd import cv2compat as G
    from monocular_visual_odometry_va4mr_amd.synth import K_KITTI as K
    rng = np.random.default_rng(3)
    R = O.rodrigues(np.array([0.01, -0.03, 0.005]))
    t = np.array([0.05, -0.02, 1.0])
    X = rng.uniform([-10, -3, 6], [10, 3, 60], (400, 3))
    P1 = K @ np.hstack([np.eye(3), np.zeros((3, 1))])
    P2 = K @ np.hstack([R, t[:, None]])
    Xh = np.c_[X, np.ones(len(X))].T
    a = P1 @ Xh
    b = P2 @ Xh
    a = (a[:2] / a[2]).T + rng.normal(size=(400, 2)) * 0.3
    b = (b[:2] / b[2]).T + rng.normal(size=(400, 2)) * 0.3
    b[:80] += rng.uniform(5, 40, (80, 2))
    a32, b32 = a.astype(np.float32), b.astype(np.float32)
    Eg, mg = G.findEssentialMat(a32, b32, K, method=G.RANSAC, prob=0.99, threshold=1)
    ok, Eo, mo = O.find_essential(a32, b32, K, 0.99, 1.0, 1000)
    assert ok and Eg is not None
    assert np.array_equal(mg.ravel(), mo)
    assert np.array_equal(Eg, Eo)
    ng, Rg, tg, _ = G.recoverPose(Eg, a32, b32, K)
    no, Ro, to, _ = O.recover_pose(Eo, a32, b32, K)
    assert ng == no and np.array_equal(Rg, Ro) and np.array_equal(tg, to)


def _oracle_init(case):
    from conftest import golden_frames, load_golden
    from oracle import vo_pipeline_oracle as V
    from monocular_visual_odometry_va4mr_amd import options as Op
    g = load_golden(case)
    fr = golden_frames(g)
    opts, boot, _ = Op.get(str(g["preset"]))
    s = V.new_state(g["K"], opts)
    V.initialize(s, fr[boot[0]], fr[boot[1]])
    return g, fr, opts, boot, s


@pytest.mark.parametrize("case", ["kitti_c2", "parking_c1", "malaga_c3", "malaga1024_c3"])
def test_bootstrap_matches_oracle(case):
    from monocular_visual_odometry_va4mr_amd.VisualOdometryPipeLine import VisualOdometryPipeLine
    g, fr, opts, boot, s = _oracle_init(case)
    vo = VisualOdometryPipeLine(g["K"], opts, max_frames=256, landmark_capacity=4096, candidate_capacity=8192)
    vo.initialization(fr[boot[0]], fr[boot[1]])
    assert vo.num_pts == [int(s.num_pts[0])]
    R_g, t_g = vo.transforms[-1]
    R_o, t_o = s.transforms[-1]
    assert np.array_equal(R_g, R_o) and np.array_equal(t_g, t_o)
    assert np.array_equal(vo.matched_landmarks, s.lm)
    assert np.array_equal(vo.matched_keypoints, s.kp)
    assert np.array_equal(vo.potential_keys, s.cand)
    assert np.array_equal(vo.potential_first_keys, s.cand_first)
    assert np.array_equal(vo.potential_transforms, s.cand_tau)
    assert np.array_equal(vo.inlier_pts_current, s.inl_pts)
    assert np.array_equal(vo.outlier_pts_current, s.outl_pts)


@pytest.mark.parametrize("case", ["kitti_c2", "parking_c1", "malaga_c3", "malaga1024_c3"])
def test_full_pipeline_ate_vs_reference(case):
    """Drop-in class on GPU vs the reference class's own run (golden fixture, produced by
    /root/reference/VisualOdometryPipeLine.py on the oracle primitives): every pose, every
    num_pts / landmark / candidate count and the snapshot arrays are bit-identical; the
    ATE (Umeyama Sim(3), reported) is therefore 0."""
    from conftest import golden_frames, load_golden
    from monocular_visual_odometry_va4mr_amd import options as Op
    from monocular_visual_odometry_va4mr_amd.VisualOdometryPipeLine import VisualOdometryPipeLine
    from monocular_visual_odometry_va4mr_amd.ate import ate
    g = load_golden(case)
    fr = golden_frames(g)
    opts, boot, _ = Op.get(str(g["preset"]))
    n = len(g["frame"])
    vo = VisualOdometryPipeLine(g["K"], opts, max_frames=max(256, n + 8), landmark_capacity=8192,
                                candidate_capacity=16384)
    vo.initialization(fr[boot[0]], fr[boot[1]])
    counts = [(len(vo.matched_landmarks), len(vo.potential_keys))]
    for i in g["frame"][1:]:
        vo.continuous_operation(fr[i])
        counts.append((len(vo.matched_landmarks), len(vo.potential_keys)))
        if f"lm_{i}" in g:
            assert np.array_equal(vo.matched_landmarks, g[f"lm_{i}"]), f"landmarks at frame {i}"
            assert np.array_equal(vo.potential_keys, g[f"cand_{i}"]), f"candidates at frame {i}"
            assert np.array_equal(vo.potential_transforms, g[f"cand_tau_{i}"]), f"frame indices at {i}"
    tr = vo.transforms[1:]
    assert len(tr) == len(g["t"])
    assert np.array_equal(np.stack([R for R, _ in tr]), g["R"])
    assert np.array_equal(np.stack([t for _, t in tr]), g["t"])
    assert vo.num_pts == [int(v) for v in g["num_pts"]]
    assert np.array_equal(np.array(counts), np.stack([g["N"], g["P"]], 1))
    est = np.array([t.ravel() for _, t in tr])
    rmse, rel = ate(est, g["t"][:, :, 0])
    assert rel == 0.0 or rel < 1e-12


@pytest.mark.parametrize("form", ["few_chains", "many_chains"])
def test_batched_bootstrap_matches_oracle_per_chain(form, launch_cus):
    """Engine.bootstrap over 6 chains with the SIFT batch forced into chunks of 2 chains
    (vo_sift_batch of 4 images, one batched BF launch and one ratio-match launch per chunk):
    every chain's state is bit-identical to the oracle's initialization on its own pair.
    Both launch forms: the split forms the small batches take (k_essential<1>,
    k_recover_count/pick, k_tri_gate/solve/append) and, with the CU threshold set to 1, the
    one-block-per-chain forms the 768-chain headline takes (k_essential<2>, k_recover_pose,
    k_triangulate)."""
    if form == "many_chains":
        launch_cus(1)
    from oracle import vo_pipeline_oracle as V
    from monocular_visual_odometry_va4mr_amd import options as Op
    from monocular_visual_odometry_va4mr_amd.engine import Engine
    from monocular_visual_odometry_va4mr_amd.features import Sift
    from monocular_visual_odometry_va4mr_amd.synth import make_sequence
    fr, K, _, _ = make_sequence("kitti", 14, seed=1)
    opts, _, _ = Op.get("kitti")
    starts = [0, 2, 4, 6, 8, 11]
    eng = Engine(K, opts, 1241, 376, batch=len(starts), ncap=4096, pcap=8192, fcap=16)
    budget = 4 * Sift.bytes_per_image(1241, 376)
    sift, m = eng.reserve_bootstrap(budget)          # reserved by the caller: kept after bootstrap
    assert sift.batch == 4 and m == 2
    eng.bootstrap(fr[starts], fr[[s + 2 for s in starts]], sift_batch_bytes=budget)
    assert eng._sift is sift
    eng.release_bootstrap()
    assert eng._sift is None
    for b, s0 in enumerate(starts):
        s = V.new_state(K, opts)
        V.initialize(s, fr[s0], fr[s0 + 2])
        e = eng.export_chain(b)
        assert e["status"] == 0
        R_g, t_g = e["transforms"][-1]
        R_o, t_o = s.transforms[-1]
        assert np.array_equal(R_g, R_o) and np.array_equal(t_g, t_o), f"chain {b}"
        for name, ref in (("landmarks", s.lm), ("keypoints", s.kp), ("cand", s.cand),
                          ("cand_first", s.cand_first), ("cand_tau", s.cand_tau)):
            assert np.array_equal(e[name], ref), f"chain {b} {name}"


def test_bootstrap_sift_capacity_marks_only_the_overflowing_chain(monkeypatch):
    """a chain whose SIFT keypoints exceed the capacity gets VO_ST_CAPACITY on the
    device (no host check inside bootstrap); the other chains of the batch are unaffected --
    bootstrap pose and state identical to an uncapped run, and they step on identically while
    the failed chain is skipped (its pose count stays); the drop-in class raises after
    initialization on such a pair."""
    from monocular_visual_odometry_va4mr_amd import _lib as L
    from monocular_visual_odometry_va4mr_amd import features as F
    from monocular_visual_odometry_va4mr_amd import options as Op
    from monocular_visual_odometry_va4mr_amd.engine import Engine
    from monocular_visual_odometry_va4mr_amd.synth import make_sequence
    from monocular_visual_odometry_va4mr_amd.VisualOdometryPipeLine import VisualOdometryPipeLine
    fr, K, _, _ = make_sequence("kitti", 14, seed=1)
    opts, _, _ = Op.get("kitti")
    starts = [0, 3, 6, 9]
    f0, f1 = fr[starts], fr[[s + 2 for s in starts]]

    def run(cap=None):
        if cap is not None:
            monkeypatch.setattr(F, "default_kp_cap", lambda w, h: cap)
        eng = Engine(K, opts, 1241, 376, batch=len(starts), ncap=8192, pcap=8192, fcap=16)
        sift, m = eng.reserve_bootstrap()
        assert m == len(starts)                       # one chunk: image rows b and B + b
        eng.bootstrap(f0, f1)
        torch.cuda.synchronize()
        raw = sift.t["counters"][:2 * len(starts), 1].cpu().numpy()     # appended before dedup
        n = np.maximum(raw[:len(starts)], raw[len(starts):])
        eng.release_bootstrap()
        for j in (3, 4):
            eng.step(fr[[s + j for s in starts]])
        torch.cuda.synchronize()
        monkeypatch.undo()
        return eng, n

    ref, n = run()
    assert (ref.statuses() == 0).all()
    order = np.argsort(n)
    assert n[order[-1]] > n[order[-2]], "needs one chain with the largest keypoint count"
    bad = int(order[-1])
    eng, _ = run(cap=int(n[order[-2]]) + 1)            # every other chain fits exactly
    st = eng.statuses()
    assert st[bad] == L.ST_CAPACITY and all(st[b] == 0 for b in range(len(starts)) if b != bad)
    assert int(eng.t["nF"][bad]) == 2                 # skipped by both steps
    for b in range(len(starts)):
        if b == bad:
            continue
        e, r = eng.export_chain(b), ref.export_chain(b)
        assert len(e["transforms"]) == len(r["transforms"]) == 4
        for (Re, te), (Rr, tr) in zip(e["transforms"], r["transforms"]):
            assert np.array_equal(Re, Rr) and np.array_equal(te, tr)
        for k in ("landmarks", "keypoints", "cand", "cand_first", "cand_tau"):
            assert np.array_equal(e[k], r[k]), (b, k)
    # the drop-in class on the overflowing pair: initialization raises (chain status)
    monkeypatch.setattr(F, "default_kp_cap", lambda w, h: int(n[order[-2]]) + 1)
    vo = VisualOdometryPipeLine(K, opts, max_frames=16, landmark_capacity=8192, candidate_capacity=8192)
    with pytest.raises(RuntimeError, match="capacity"):
        vo.initialization(f0[bad], f1[bad])
