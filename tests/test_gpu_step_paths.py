"""The step's launch forms give the same state: the engine default (vo_track_lk +
vo_filter_pnp_triangulate), tracking with its own filtering launch (vo_track +
vo_pnp_triangulate, VO_COMPACT_IN_TRACK=1), the separate PnP / triangulation calls
(vo_track + vo_pnp + vo_triangulate, fuse_pnp_tri = False) and the latency stages on a
stream of their own (VO_PRIO_LATENCY=1), eager and replayed from a hipGraph -- every C-ABI
path of the step, at both sides of the launch-shape threshold (vo_set_launch_cus)."""
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
    if form.startswith("prio_latency"):            # PnP + finish on a high-priority stream of their own
        monkeypatch.setenv("VO_PRIO_LATENCY", "1")
    else:
        monkeypatch.delenv("VO_PRIO_LATENCY", raising=False)
    eng = Engine(K, opts, 1241, 376, batch=len(starts), ncap=4096, pcap=8192, fcap=16)
    if form == "split":
        eng.fuse_pnp_tri = False
    eng.bootstrap(frames[starts], frames[[s + 2 for s in starts]])
    snaps = []
    graph = form.endswith("graph")
    if graph:
        eng.capture_step()
    for j in range(n_steps):
        f = frames[[s + 3 + j for s in starts]]
        if graph:
            eng.step_graph(f)
        else:
            eng.step(f)
        torch.cuda.synchronize()
        snaps.append({k: eng.t[k].cpu().numpy().copy() for k in KEYS})
    return snaps


@pytest.mark.parametrize("cus", [0, 1])
def test_step_launch_forms_agree(monkeypatch, launch_cus, cus):
    """cus = 1: every launch takes the many-chains form (k_pnp_tri / k_pnp_fused at 2 waves
    per EU, the one-block triangulation) -- the forms of the 768-chain headline; the default
    run (cus = 0, the device's own count) takes the unconstrained builds.  Both are compared
    with the same reference run (default form, default threshold)."""
    from monocular_visual_odometry_va4mr_amd import options as Op
    from monocular_visual_odometry_va4mr_amd.synth import make_sequence
    fr, K, _, _ = make_sequence("kitti", 14, seed=1)
    opts, _, _ = Op.get("kitti")
    frames = torch.from_numpy(np.ascontiguousarray(fr)).cuda()
    starts = [0, 1, 3]
    ref = _run(frames, starts, K, opts, 7, "default", monkeypatch)
    assert (ref[-1]["status"] == 0).all()
    launch_cus(cus)
    forms = ("default", "compact_in_track", "split", "prio_latency", "graph", "prio_latency_graph")
    runs = {f: _run(frames, starts, K, opts, 7, f, monkeypatch) for f in forms}
    for f in forms:
        for j, (a, b) in enumerate(zip(ref, runs[f])):
            for k in KEYS:
                assert np.array_equal(a[k], b[k]), f"{f}: step {j} {k}"


def test_prefetch_graph_and_host_frames_mixed():
    """a pending next-frames pyramid build (step(..., next_frames=...)) followed by a
    graph replay, a pyramid rebuild or host (numpy) frames must give the state of plain eager
    steps; the captured step reads device frames in place (frame slot) and host frames through
    its own buffer."""
    from monocular_visual_odometry_va4mr_amd import options as Op
    from monocular_visual_odometry_va4mr_amd.engine import Engine
    from monocular_visual_odometry_va4mr_amd.synth import make_sequence
    fr, K, _, _ = make_sequence("kitti", 14, seed=1)
    opts, _, _ = Op.get("kitti")
    frames = torch.from_numpy(np.ascontiguousarray(fr)).cuda()
    starts = [0, 2]
    f = lambda j: frames[[s + 3 + j for s in starts]].contiguous()

    def fresh():
        e = Engine(K, opts, 1241, 376, batch=len(starts), ncap=4096, pcap=8192, fcap=16)
        e.bootstrap(frames[starts], frames[[s + 2 for s in starts]])
        return e

    ref = fresh()
    ref_snaps = []
    for j in range(8):
        ref.step(f(j))
        torch.cuda.synchronize()
        ref_snaps.append({k: ref.t[k].cpu().numpy().copy() for k in KEYS})
    eng = fresh()
    eng.capture_step()
    keep = [f(j) for j in range(8)]          # the same tensors: a prefetch is keyed on them
    plan = [("eager_next", 1), ("graph", None), ("eager_next", 3), ("eager", None), ("graph_host", None),
            ("eager_next", 6), ("graph", None), ("eager", None)]
    for j, (how, nxt) in enumerate(plan):
        if how == "eager_next":
            eng.step(keep[j], next_frames=keep[nxt])
        elif how == "eager":
            eng.step(keep[j])
        elif how == "graph":
            eng.step_graph(keep[j])
        else:
            eng.step_graph(keep[j].cpu().numpy())
        torch.cuda.synchronize()
        for k in KEYS:
            assert np.array_equal(ref_snaps[j][k], eng.t[k].cpu().numpy()), f"step {j} ({how}): {k}"
    assert (ref_snaps[-1]["status"] == 0).all()
