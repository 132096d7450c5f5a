#!/usr/bin/env python3
"""Pyramid + Scharr build (vo_pyr_build) of B KITTI-size frames alone on the GPU: ms per build,
per-chain cost and the algorithmic HBM rate (frame read, every level's bytes and int16 (dx, dy)
pairs written, every pyrDown level's source read).  Run under rocprofv3 --kernel-trace --stats
for the per-level split.
usage: python tools/pyr_bench.py [B ...]   (default 16 384 768)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from monocular_visual_odometry_va4mr_amd import options as Op  # noqa: E402
from monocular_visual_odometry_va4mr_amd.engine import Engine  # noqa: E402
from monocular_visual_odometry_va4mr_amd.synth import Renderer  # noqa: E402


def main():
    Bs = [int(a) for a in sys.argv[1:]] or [16, 384, 768]
    dev = torch.device("cuda", 0)
    opts, _, _ = Op.get("kitti")
    rend = Renderer("kitti", seed=1, device=dev)
    W, H = rend.W, rend.H
    for B in Bs:
        eng = Engine(rend.K, opts, W, H, batch=B, device=dev, ncap=16, pcap=16, fcap=4)
        g = torch.Generator(device=dev).manual_seed(B)
        frames = torch.randint(0, 256, (B, H, W), dtype=torch.uint8, device=dev, generator=g)
        for _ in range(3):
            eng.build_pyramid(frames, 0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record()
        for r in range(reps):
            eng.build_pyramid(frames, r & 1)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        d = eng.dims
        lw, lh = list(d.lvl_w), list(d.lvl_h)
        nlev = d.nlev
        per_chain = W * H + sum(5 * lw[l] * lh[l] for l in range(nlev)) + sum(lw[l - 1] * lh[l - 1] for l in range(1, nlev))
        gbs = B * per_chain / (ms * 1e-3) / 1e9
        print(json.dumps({"B": B, "levels": nlev, "ms_per_build": round(ms, 4), "us_per_chain": round(ms * 1e3 / B, 3),
                          "algorithmic_bytes_per_chain": per_chain, "GB_per_s": round(gbs, 1)}), flush=True)
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
