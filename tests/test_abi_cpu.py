"""CPU-side checks of the C ABI and host logic (no GPU calls)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from monocular_visual_odometry_va4mr_amd import _lib as L


def test_library_exports_every_declared_symbol():
    if not os.path.exists(L.LIB_PATH):
        L.build()
    lib = ctypes.CDLL(L.LIB_PATH)          # loads without a GPU
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True).stdout
    defined = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    declared = L.exported_symbols()
    assert len(declared) >= 20
    missing = [s for s in declared if s not in defined]
    assert not missing, missing
    for s in declared:
        assert hasattr(lib, s)


def test_struct_layouts_match_header():
    """ctypes mirrors of vo_dims / vo_opts / vo_state / vo_sift_buf have the C sizes."""
    src = r'''
    #include <stdio.h>
    #include <stddef.h>
    #include "vo_hip.h"
    int main(void) {
        printf("%zu %zu %zu %zu %zu %zu\n", sizeof(vo_dims), sizeof(vo_opts), sizeof(vo_state),
               sizeof(vo_sift_buf), offsetof(vo_dims, work_stride), offsetof(vo_opts, pnp_iters));
        return 0;
    }'''
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    tmp = "/tmp/vo_abi_layout"
    with open(tmp + ".c", "w") as f:
        f.write(src)
    subprocess.run(["gcc", "-I", inc, tmp + ".c", "-o", tmp], check=True)
    vals = [int(v) for v in subprocess.run([tmp], capture_output=True, text=True).stdout.split()]
    assert vals[0] == ctypes.sizeof(L.VoDims)
    assert vals[1] == ctypes.sizeof(L.VoOpts)
    assert vals[2] == ctypes.sizeof(L.VoState)
    assert vals[3] == ctypes.sizeof(L.VoSiftBuf)
    assert vals[4] == L.VoDims.work_stride.offset
    assert vals[5] == L.VoOpts.pnp_iters.offset


def test_no_gpu_means_loud_failure(monkeypatch):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from monocular_visual_odometry_va4mr_amd.engine import Engine
    from monocular_visual_odometry_va4mr_amd import options as O
    opts, _, _ = O.get("kitti")
    with pytest.raises(RuntimeError):
        Engine(np.eye(3), opts, 64, 48)


def test_pyramid_levels_match_oracle():
    from oracle import _olib as O
    from monocular_visual_odometry_va4mr_amd.engine import pyr_max_level
    for w, h, ml in [(1241, 376, 5), (640, 480, 10), (800, 600, 10), (1024, 768, 10), (1920, 1080, 5), (31, 20, 3)]:
        assert pyr_max_level(w, h, (15, 15), ml) == O.pyr_maxlevel(w, h, (15, 15), ml)


def test_options_match_reference_driver():
    from monocular_visual_odometry_va4mr_amd import options as O
    k, boot, last = O.get("kitti")
    assert boot == (0, 2) and last == 2761 and k["PnP_error"] == 8 and k["maxLevel"] == 5
    p, boot, last = O.get("parking")
    assert boot == (0, 6) and last == 598 and p["criteria"][2] == 0.02 and p["max_dist_landmarks"] == 50
    m, boot, last = O.get("malaga")
    assert boot == (0, 6) and last == 2120 and m["feature_quality_level"] == 0.03 and m["min_dist_landmarks"] == 0


def test_ate_umeyama_recovers_sim3():
    from monocular_visual_odometry_va4mr_amd.ate import ate
    rng = np.random.default_rng(0)
    ref = np.cumsum(rng.normal(size=(50, 3)), 0)
    a = 0.3
    R = np.array([[np.cos(a), -np.sin(a), 0], [np.sin(a), np.cos(a), 0], [0, 0, 1]])
    est = (2.5 * (R @ ref.T)).T + np.array([1, 2, 3])
    rmse, rel = ate(est, ref)
    assert rmse < 1e-9 and rel < 1e-10


def test_synth_is_deterministic_and_textured():
    from monocular_visual_odometry_va4mr_amd.synth import make_sequence
    a, K, R, c = make_sequence("parking", 2, seed=7)
    b, _, _, _ = make_sequence("parking", 2, seed=7)
    assert np.array_equal(a, b) and a.dtype == np.uint8 and a.shape == (2, 480, 640)
    assert a.std() > 15
    assert np.allclose(c[1] - c[0], [0, 0, 1], atol=0.01)


class _StatusEngine:
    """Stand-in for a one-chain Engine that only reports a scripted (status, inliers) per frame."""

    def __init__(self, script):
        self.script = list(script)

    def step(self, frames):
        pass

    step_graph = step

    def status_word(self, in_graph=False):
        return self.script.pop(0)


@pytest.mark.parametrize("crash,exc", [(L.ST_GFTT_NONE, AttributeError), (L.ST_GFTT_ONE, IndexError),
                                       (L.ST_NOT_ENOUGH_KP, ValueError), (L.ST_PNP_FAILED, ValueError)])
def test_dropin_ring_appends_before_feature_adding_crash(crash, exc):
    """VisualOdometryPipeLine.py:360-369: the 20-entry ring gets the frame's inlier count after
    PnP succeeded and before feature_adding, so a goodFeaturesToTrack crash (:256) leaves it
    appended; a PnP failure (:352, :358) raises before the ring is touched."""
    from monocular_visual_odometry_va4mr_amd.VisualOdometryPipeLine import VisualOdometryPipeLine
    from monocular_visual_odometry_va4mr_amd import options as O
    opts, _, _ = O.get("kitti")
    vo = VisualOdometryPipeLine(np.eye(3), opts)
    script = [(L.ST_OK, 100 + i) for i in range(22)] + [(crash, 77)]
    vo._eng = _StatusEngine(script)
    vo._boot_done = True
    img = np.zeros((4, 4), np.uint8)
    for _ in range(22):
        vo.continuous_operation(img)
    assert vo.num_tracked_landmarks_list == list(range(102, 122))
    with pytest.raises(exc):
        vo.continuous_operation(img)
    appended = crash in (L.ST_GFTT_NONE, L.ST_GFTT_ONE)
    assert vo.num_tracked_landmarks_list == list(range(103 if appended else 102, 122)) + ([77] if appended else [])
