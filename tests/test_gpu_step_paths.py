"""The step's three launch forms give the same state: the engine default (vo_track_lk +
vo_filter_pnp_triangulate), tracking with its own filtering launch (vo_track +
vo_pnp_triangulate, VO_COMPACT_IN_TRACK=1) and the separate PnP / triangulation calls
(vo_track + vo_pnp + vo_triangulate, fuse_pnp_tri = False) -- every C-ABI path of the step."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

KEYS = ("status", "nL", "nC", "nF", "lm_X", "lm_kp", "c_kp", "c_first", "c_tau", "pose_R", "pose_t",
        "num_pts", "nInl")


def _run(frames, starts, K, opts, n_steps, form, monkeypatch):
    from monocular_visual_odometry_va4mr_amd.engine import Engine
    if form == "compact_in_track":
        monkeypatch.setenv("VO_COMPACT_IN_TRACK", "1")
    else:
        monkeypatch.delenv("VO_COMPACT_IN_TRACK", raising=False)
    eng = Engine(K, opts, 1241, 376, batch=len(starts), ncap=4096, pcap=8192, fcap=16)
    if form == "split":
        eng.fuse_pnp_tri = False
    eng.bootstrap(frames[starts], frames[[s + 2 for s in starts]])
    snaps = []
    for j in range(n_steps):
        eng.step(frames[[s + 3 + j for s in starts]])
        torch.cuda.synchronize()
        snaps.append({k: eng.t[k].cpu().numpy().copy() for k in KEYS})
    return snaps


def test_step_launch_forms_agree(monkeypatch):
    from monocular_visual_odometry_va4mr_amd import options as Op
    from monocular_visual_odometry_va4mr_amd.synth import make_sequence
    fr, K, _, _ = make_sequence("kitti", 14, seed=1)
    opts, _, _ = Op.get("kitti")
    frames = torch.from_numpy(np.ascontiguousarray(fr)).cuda()
    starts = [0, 1, 3]
    runs = {f: _run(frames, starts, K, opts, 7, f, monkeypatch) for f in ("default", "compact_in_track", "split")}
    ref = runs["default"]
    assert (ref[-1]["status"] == 0).all()
    for f in ("compact_in_track", "split"):
        for j, (a, b) in enumerate(zip(ref, runs[f])):
            for k in KEYS:
                assert np.array_equal(a[k], b[k]), f"{f}: step {j} {k}"
