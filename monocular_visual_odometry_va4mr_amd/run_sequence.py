"""Sharded run of one sequence across chains and GPUs, end to end.

    python -m monocular_visual_odometry_va4mr_amd.run_sequence --preset kitti --frames 4541 \
        --shards-per-gpu 8 [--overlap 30] [--out poses.txt]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        -m monocular_visual_odometry_va4mr_amd.run_sequence ...

The sequence is cut into N*B contiguous shards with overlap (shards.plan_shards); rank r
owns a block of B shards and runs them as the B chains of one Engine: bootstrap at
[s, s+gap] (main.py:18,48,78), then continuous_operation on the following frames, feeding
every chain its own next frame each step.  When all ranks are done, the per-chain poses are
all-gathered to rank 0 (the one collective; RCCL on GPUs), which stitches the shards with
Sim(3) fits on the overlap frames and evaluates against ground truth.  Frames come from the
seeded renderer (synth.py), rendered on the GPU per step.
"""
from __future__ import annotations

import argparse
import json
import os
import time

import numpy as np
import torch

from . import evaluation as Ev
from . import options as Op
from . import shards as Sh
from .engine import Engine
from .synth import Renderer, poses


def run(preset: str, n_frames: int, shards_per_rank: int, overlap: int = 30, seed: int = 1, device=None,
        rank: int = 0, world: int = 1, out_path: str | None = None) -> dict | None:
    dev = torch.device(device or "cuda")
    opts, (b0, b1), _ = Op.get(preset)
    gap = b1 - b0
    plan = Sh.plan_shards(n_frames, world * shards_per_rank, gap, overlap)
    mine = Sh.rank_shards(plan, rank, world)
    B = len(mine)
    rend = Renderer(preset, seed=seed, device=dev)
    Rs, cs = poses(n_frames, rend.p)
    max_f = max(s.end - s.boot1 + 1 for s in plan)
    eng = Engine(rend.K, opts, rend.W, rend.H, batch=B, device=dev, ncap=16384, pcap=16384, fcap=max_f + 8)

    def frames_at(ids):
        ids = [min(int(i), n_frames - 1) for i in ids]
        return rend.render_batch(ids, Rs[ids], cs[ids])

    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    eng.bootstrap(frames_at([s.start for s in mine]), frames_at([s.boot1 for s in mine]))
    n_steps = max(s.n_steps for s in mine)
    t_step = 0.0
    for j in range(n_steps):
        # chains whose shard has ended keep re-reading their last frame (zero motion);
        # their extra poses are dropped below
        fr = frames_at([min(s.boot1 + 1 + j, s.end - 1) for s in mine])
        torch.cuda.synchronize(dev)
        ts = time.perf_counter()
        eng.step(fr)
        torch.cuda.synchronize(dev)
        t_step += time.perf_counter() - ts
    wall = time.perf_counter() - t0
    packed = Sh.pack_poses(eng.t["pose_R"], eng.t["pose_t"], eng.t["nF"], eng.dims.fcap)
    allp = Sh.gather_poses(packed)
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        st_all = [torch.empty_like(eng.t["status"]) for _ in range(world)]
        dist.all_gather(st_all, eng.t["status"])
        statuses = torch.cat(st_all).cpu().numpy()
        tt = torch.tensor([t_step, wall], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_step, wall = (float(v) for v in tt.cpu())
    else:
        statuses = eng.t["status"].cpu().numpy()
    if allp is None:
        return None
    allp = allp.cpu().numpy()
    centres, ok_shards, ok_centres = [], [], []
    for s, chain in zip(plan, allp):
        c = Sh.unpack_centres(chain)[: s.end - s.boot1 + 1]
        centres.append(c)
    for s, c, st in zip(plan, centres, statuses):
        if st == 0 and len(c) == s.end - s.boot1 + 1:
            ok_shards.append(s)
            ok_centres.append(c)
    stitched = Sh.stitch(ok_shards, ok_centres) if ok_shards else None
    rep = Ev.shard_report(ok_shards, ok_centres, cs, stitched)
    frames_done = sum(s.n_steps for s in plan)
    out = {
        "preset": preset, "frames": n_frames, "shards": len(plan), "gpus": world, "chains_per_gpu": shards_per_rank,
        "overlap": overlap, "shards_ok": len(ok_shards),
        "shard_status": {str(int(k)): int(v) for k, v in zip(*np.unique(statuses, return_counts=True))},
        "step_frames_per_s": round(frames_done / max(t_step, 1e-9), 1),
        "wall_s": round(wall, 2), "step_s": round(t_step, 3),
        "shard_ate_rel_max": max((p["ate_rel"] for p in rep["shards"]), default=None),
        "stitched": rep.get("stitched"),
    }
    if out_path and stitched is not None:
        keep = ~np.isnan(stitched[:, 0])
        np.savetxt(out_path, np.c_[np.nonzero(keep)[0], stitched[keep]], fmt=["%d", "%.9f", "%.9f", "%.9f"])
    out["_centres"] = centres
    out["_plan"] = plan
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="kitti")
    ap.add_argument("--frames", type=int, default=600)
    ap.add_argument("--shards-per-gpu", type=int, default=8)
    ap.add_argument("--overlap", type=int, default=30)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default=None, help="write the stitched positions (frame x y z)")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    res = run(args.preset, args.frames, args.shards_per_gpu, args.overlap, args.seed, dev, rank, world, args.out)
    if res is not None:
        print(json.dumps({k: v for k, v in res.items() if not k.startswith("_")}))
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
