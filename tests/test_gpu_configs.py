"""Parity at the BASELINE configurations beyond C2, through the C ABI:

C5  synthetic 1920x1080, GFTT maxCorners 8192 / qualityLevel 0.01 / minDistance 5 (~8k
    corners per frame), KLT on every tracked point (~12.7k), one full engine step
C3  Malaga 1024x768: SIFT on consecutive frames + batched BF 2-NN (the MFMA path), and the
    reference class's own run on that sequence (golden malaga1024_c3)

Every comparison is bit-exact against the CPU oracle on the same inputs."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def hd_frames():
    from monocular_visual_odometry_va4mr_amd.synth import make_sequence
    fr, K, _, _ = make_sequence("hd1080", 8, seed=3)
    return fr, K


def _engine(K, W, H, preset="hd1080", **kw):
    from monocular_visual_odometry_va4mr_amd import options as Op
    from monocular_visual_odometry_va4mr_amd.engine import Engine
    opts, _, _ = Op.get(preset)
    opts.update(kw)
    return Engine(K, opts, W, H, batch=1, ncap=32768, pcap=32768, fcap=64), opts


def test_c5_gftt_bitexact(hd_frames):
    from oracle import _olib as O
    fr, K = hd_frames
    eng, opts = _engine(K, 1920, 1080)
    eng.build_pyramid(fr[1], 0)
    assert eng.lib.vo_gftt(eng._pd, eng._po, eng._ps, 0, eng.stream) == 0
    torch.cuda.synchronize()
    n = int(eng.t["nCorners"][0])
    got = eng.t["corners"][0, :n].cpu().numpy()
    ref = O.gftt(fr[1], 8192, 0.01, 5, 3)
    assert n > 6000
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("harris,bs", [(True, 3), (False, 5), (True, 7)])
def test_c5_gftt_harris_blocksize_bitexact(hd_frames, harris, bs):
    """C5 size with feature_use_harris / feature_block_size (main.py:32-33 -> VOPL:256)."""
    from oracle import _olib as O
    fr, K = hd_frames
    q = 0.001 if harris else 0.01
    eng, opts = _engine(K, 1920, 1080, feature_use_harris=harris, feature_block_size=bs, feature_quality_level=q)
    eng.build_pyramid(fr[1], 0)
    assert eng.lib.vo_gftt(eng._pd, eng._po, eng._ps, 0, eng.stream) == 0
    torch.cuda.synchronize()
    n = int(eng.t["nCorners"][0])
    got = eng.t["corners"][0, :n].cpu().numpy()
    ref = O.gftt(fr[1], 8192, q, 5, bs, use_harris=harris)
    assert n > 4000
    assert np.array_equal(got, ref)


def test_gftt_capacity_is_reported_not_truncated(hd_frames):
    """More corners wanted than the engine holds (maxCorners 0 = unlimited; the corner buffer is
    8,192): the selection reports the overflow (nCorners = -1, which k_add_finish turns into
    VO_ST_CAPACITY) instead of returning a silently truncated list."""
    from oracle import _olib as O
    fr, K = hd_frames
    eng, opts = _engine(K, 1920, 1080, feature_max_corners=0, feature_quality_level=0.001, feature_min_dist=1)
    assert eng.dims.mcap == 8192
    eng.build_pyramid(fr[1], 0)
    assert eng.lib.vo_gftt(eng._pd, eng._po, eng._ps, 0, eng.stream) == 0
    torch.cuda.synchronize()
    ref = O.gftt(fr[1], 0, 0.001, 1, 3)
    assert len(ref) > 8192
    assert int(eng.t["nCorners"][0]) == -1


def test_c5_lk_bitexact(hd_frames):
    """KLT on ~12.7k points at 1080p: GFTT corners of frame 0 plus jittered copies (the
    candidate + landmark load of a C5 step), tracked 0 -> 1."""
    from oracle import _olib as O
    fr, K = hd_frames
    eng, opts = _engine(K, 1920, 1080)
    c = O.gftt(fr[0], 8192, 0.01, 5, 3)
    rng = np.random.default_rng(5)
    jit = (c[:4700] + rng.uniform(-3, 3, (min(4700, len(c)), 2))).astype(np.float32)
    pts = np.concatenate([c, jit]).astype(np.float32)
    n = len(pts)
    assert n > 12000
    eng.build_pyramid(fr[0], 0)
    eng.build_pyramid(fr[1], 1)
    dpts = torch.from_numpy(pts).cuda().reshape(1, n, 2)
    cnt = torch.tensor([n], dtype=torch.int32, device="cuda")
    out = torch.zeros(1, n, 2, device="cuda")
    st = torch.zeros(1, n, dtype=torch.uint8, device="cuda")
    err = torch.zeros(1, n, device="cuda")
    rc = eng.lib.vo_lk_points(eng._pd, eng._po, eng._ps, 0, C.c_void_p(dpts.data_ptr()), C.c_void_p(cnt.data_ptr()),
                              n, C.c_void_p(out.data_ptr()), C.c_void_p(st.data_ptr()), C.c_void_p(err.data_ptr()),
                              eng.stream)
    assert rc == 0
    torch.cuda.synchronize()
    ro, rs, re = O.lk(fr[0], fr[1], pts, tuple(opts["winSize"]), opts["maxLevel"], opts["criteria"])
    assert np.array_equal(st.cpu().numpy()[0], rs)
    assert np.array_equal(out.cpu().numpy()[0], ro)
    m = rs == 1
    assert m.mean() > 0.5
    assert np.array_equal(err.cpu().numpy()[0][m], re[m])


def test_c5_bootstrap_and_step_bitexact(hd_frames):
    """C5 end to end on one chain: GPU initialization (SIFT at 1080p, BF, E-RANSAC,
    recoverPose, triangulation) and two continuous_operation steps vs the oracle."""
    from oracle import vo_pipeline_oracle as V
    fr, K = hd_frames
    eng, opts = _engine(K, 1920, 1080)
    s = V.new_state(K, opts)
    V.initialize(s, fr[0], fr[2])
    eng.bootstrap(fr[0][None], fr[2][None])
    e = eng.export_chain(0)
    assert e["status"] == 0
    for name, ref in (("landmarks", s.lm), ("cand", s.cand), ("cand_first", s.cand_first)):
        assert np.array_equal(e[name], ref), f"bootstrap {name}"
    for i in (3, 4):
        V.step(s, fr[i])
        eng.step(fr[i][None])
        e = eng.export_chain(0)
        assert e["status"] == 0
        R_g, t_g = e["transforms"][-1]
        R_o, t_o = s.transforms[-1]
        assert np.array_equal(R_g, R_o) and np.array_equal(t_g, t_o), f"pose at frame {i}"
        for name, ref in (("landmarks", s.lm), ("keypoints", s.kp), ("cand", s.cand),
                          ("cand_first", s.cand_first), ("cand_tau", s.cand_tau)):
            assert np.array_equal(e[name], ref), f"{name} at frame {i}"
        assert int(eng.t["nCorners"][0]) > 6000


def test_c5_sift_capped_and_bf_bitexact(hd_frames):
    """C5's "SIFT capped at the best 8192 + BF 8192^2" on two consecutive 1920x1080 frames:
    SIFT_create(nfeatures=8192) batched over both frames (vo_sift_batch; retainBest in
    libstdc++'s nth_element / partition order, k_sift_retain_best), then the 8192 x 8192 2-NN
    on MFMA (vo_bf_knn2_batch) -- keypoints, descriptors, indices and distances bit for bit
    against O.sift(nfeatures=8192) + O.bf_knn2.  The uncapped detector finds > 8192 keypoints
    on both frames, so the cap really selects."""
    from oracle import _olib as O
    from monocular_visual_odometry_va4mr_amd.features import Sift, bf_knn2_batch
    fr, _ = hd_frames
    imgs = torch.from_numpy(np.ascontiguousarray(fr[:2])).cuda()
    full = Sift(1920, 1080, "cuda", batch=2)
    _, _, n_full = full.run_batch(imgs)
    assert (n_full.cpu().numpy() > 8192).all()
    del full
    sift = Sift(1920, 1080, "cuda", batch=2, nfeatures=8192)
    kp, desc, n = sift.run_batch(imgs)
    assert not sift.overflowed(2)
    n = n.cpu().numpy()
    ref = []
    for b in range(2):
        ko, do = O.sift(fr[b], nfeatures=8192)
        assert n[b] == len(ko) >= 8192
        assert np.array_equal(kp[b, :n[b]].cpu().numpy(), ko), f"frame {b} keypoints"
        assert np.array_equal(desc[b, :n[b]].cpu().numpy(), do), f"frame {b} descriptors"
        ref.append(do)
    nd = torch.as_tensor(n, dtype=torch.int32, device="cuda")
    idx2, dist2 = bf_knn2_batch(desc[:1], nd[:1], desc[1:2], nd[1:2])
    ei, ed = O.bf_knn2(ref[0], ref[1])
    assert np.array_equal(idx2[0, :n[0]].cpu().numpy(), ei)
    assert np.array_equal(dist2[0, :n[0]].cpu().numpy(), ed)


def test_c3_sift_batched_match_bitexact():
    """C3 1024x768: SIFT of 5 consecutive frames, the 4 consecutive pairs matched in one
    vo_bf_knn2_batch launch, each against O.sift + O.bf_knn2."""
    from oracle import _olib as O
    from monocular_visual_odometry_va4mr_amd.features import Sift, bf_knn2_batch
    from monocular_visual_odometry_va4mr_amd.synth import make_sequence
    fr, _, _, _ = make_sequence("malaga1024", 5, seed=2)
    sift = Sift(1024, 768, "cuda")
    D = torch.zeros((5, sift.kp_cap, 128), dtype=torch.float32, device="cuda")
    N = torch.zeros(5, dtype=torch.int32, device="cuda")
    ref = []
    for i in range(5):
        kp, desc, n = sift.run(torch.from_numpy(np.ascontiguousarray(fr[i])).cuda())
        D[i].copy_(desc)
        N[i:i + 1].copy_(n)
        ko, do = O.sift(fr[i])
        assert int(n) == len(ko) > 1000
        assert np.array_equal(kp[:len(ko)].cpu().numpy(), ko)
        assert np.array_equal(desc[:len(ko)].cpu().numpy(), do)
        ref.append(do)
    idx2, dist2 = bf_knn2_batch(D[:-1], N[:-1], D[1:], N[1:])
    idx2, dist2 = idx2.cpu().numpy(), dist2.cpu().numpy()
    for p in range(4):
        ei, ed = O.bf_knn2(ref[p], ref[p + 1])
        nq = len(ref[p])
        assert np.array_equal(idx2[p, :nq], ei) and np.array_equal(dist2[p, :nq], ed), f"pair {p}"
