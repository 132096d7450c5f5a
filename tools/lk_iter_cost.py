"""Marginal cost of one LK iteration (k_lk_w), loaded and unloaded (diagnostics; results differ
from the reference when the iteration cap is changed -- timing only).

    python tools/lk_iter_cost.py [B ...]
    python tools/lk_iter_cost.py --save DIR [B ...]     (also write the tracked points)
    VO_HIP_LIB=... python tools/lk_iter_cost.py --load DIR [B ...]   (time another build of
        libvo_hip.so on the saved points: no bootstrap or step runs through it)

For each batch B: B chains of the C2 workload are bootstrapped and stepped a few frames, then
their landmark + candidate points are tracked from pyr[prev] to pyr[cur] with vo_lk_points
(no state change) under criteria counts 1, 2, 3, 5, 50.  The kernel time (HIP events, median
of 5) against the mean iteration count gives the per-iteration slope and the fixed per-point
cost (staging, tensor, err)."""
from __future__ import annotations

import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from monocular_visual_odometry_va4mr_amd import options as Op  # noqa: E402
from monocular_visual_odometry_va4mr_amd.engine import Engine  # noqa: E402
from monocular_visual_odometry_va4mr_amd.synth import Renderer  # noqa: E402


def _prepare(B, dev, opts, gap, rend, gt, save_dir=None, load_dir=None):
    n_after = 4
    window = gap + 1 + n_after
    starts = [min((g * bench.SEQ_LEN) // max(B, 1), bench.SEQ_LEN - window) for g in range(B)]
    frames = bench.render_windows(rend, gt, starts, gap, n_after, dev)
    eng = Engine(rend.K, opts, rend.W, rend.H, batch=B, device=dev, ncap=16384, pcap=16384, fcap=64)
    if load_dir is None:
        eng.bootstrap(frames[0], frames[1])
        for j in range(2, 2 + n_after - 1):
            eng.step(frames[j])
        # next frame's pyramid into pyr[1 - prev]; track landmarks + candidates prev -> cur
        eng.build_pyramid(frames[2 + n_after - 1], 1 - eng.prev)
        torch.cuda.synchronize()
        nL, nC = eng.t["nL"].long(), eng.t["nC"].long()
        cap = int((nL + nC).max())
        pts = torch.zeros((B, cap, 2), dtype=torch.float32, device=dev)
        for b in range(B):
            a, c = int(nL[b]), int(nC[b])
            pts[b, :a] = eng.t["lm_kp"][b, :a]
            pts[b, a:a + c] = eng.t["c_kp"][b, :c]
        cnt = (nL + nC).to(torch.int32)
        if save_dir:
            np.savez(os.path.join(save_dir, f"lk_pts_{B}.npz"), pts=pts.cpu().numpy(), cnt=cnt.cpu().numpy(),
                     prev=eng.prev)
    else:
        z = np.load(os.path.join(load_dir, f"lk_pts_{B}.npz"))
        pts = torch.from_numpy(z["pts"]).to(dev)
        cnt = torch.from_numpy(z["cnt"]).to(dev)
        cap = pts.shape[1]
        eng.prev = int(z["prev"])
        eng.build_pyramid(frames[2 + n_after - 2], eng.prev)
        eng.build_pyramid(frames[2 + n_after - 1], 1 - eng.prev)
        torch.cuda.synchronize()
    return eng, frames, pts, cnt, cap


def main():
    argv = sys.argv[1:]
    save_dir = load_dir = None
    if "--save" in argv:
        i = argv.index("--save")
        save_dir = argv[i + 1]
        argv = argv[:i] + argv[i + 2:]
    if "--load" in argv:
        i = argv.index("--load")
        load_dir = argv[i + 1]
        argv = argv[:i] + argv[i + 2:]
    counts = (1, 2, 3, 5, 8, 50) if load_dir is None else (1, 50)
    Bs = [int(a) for a in argv] or [1, 384]
    dev = torch.device("cuda", 0)
    opts, (b0, b1), _ = Op.get("kitti")
    gap = b1 - b0
    rend = Renderer("kitti", seed=1, device=dev)
    gt = bench.StagePoses(bench.SEQ_LEN, rend.p)
    for B in Bs:
        eng, frames, pts, cnt, cap = _prepare(B, dev, opts, gap, rend, gt, save_dir, load_dir)
        out = torch.zeros_like(pts)
        st = torch.zeros((B, cap), dtype=torch.uint8, device=dev)
        err = torch.zeros((B, cap), dtype=torch.float32, device=dev)
        npts = int(cnt.sum())
        res = []
        for count in counts:
            eng.opts.crit_count = count
            ts = []
            for _ in range(6):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                rc = eng.lib.vo_lk_points(eng._pd, eng._po, eng._ps, eng.prev, C.c_void_p(pts.data_ptr()),
                                          C.c_void_p(cnt.data_ptr()), cap, C.c_void_p(out.data_ptr()),
                                          C.c_void_p(st.data_ptr()), C.c_void_p(err.data_ptr()), eng.stream)
                e1.record()
                assert rc == 0
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            res.append({"count": count, "ms": round(float(np.median(ts[1:])), 4),
                        "tracked": int(st.sum())})
        eng.opts.crit_count = int(opts["criteria"][1])
        print(json.dumps({"lib": os.path.basename(os.environ.get("VO_HIP_LIB", "libvo_hip.so")), "B": B,
                          "points": npts, "levels": eng.dims.nlev, "runs": res}), flush=True)
        del eng, frames
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
