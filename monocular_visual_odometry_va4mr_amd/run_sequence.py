"""Sharded run of one sequence across chains and GPUs, end to end.

    python -m monocular_visual_odometry_va4mr_amd.run_sequence --preset kitti --frames 4541 \
        --shards-per-gpu 8 [--overlap 15] [--out poses.txt]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        -m monocular_visual_odometry_va4mr_amd.run_sequence ...

The sequence is cut into N*B contiguous shards with overlap (shards.plan_shards); rank r
owns a block of B shards and runs them as the B chains of one Engine: bootstrap at
[s, s+gap] (main.py:18,48,78), then continuous_operation on the following frames, feeding
every chain its own next frame each step.  When all ranks are done, the per-chain poses and
statuses are all-gathered to rank 0 (the one collective; RCCL on GPUs), which stitches the
surviving shards with Sim(3) fits on the overlap frames (a shard that cannot be chained opens
a new segment and is reported as a coverage break) and evaluates against ground truth and,
when given, against the reference CPU path's per-shard trajectories (§8e parity).  Frames
come from the seeded renderer (synth.py), rendered into device memory before the run.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import time

import numpy as np
import torch

from . import evaluation as Ev
from . import options as Op
from . import shards as Sh


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def default_groups(chains: int) -> int:
    """Stream groups for a rank's chains (run's ``groups``): one engine up to 16 chains
    (latency-bound: a second stream only adds a queue hop), two above (measured,
    tools/seq_sweep.py)."""
    return 1 if chains <= 16 else 2


def run(preset: str, n_frames: int, shards_per_rank: int, overlap: int = 30, seed: int = 1, device=None,
        rank: int = 0, world: int = 1, out_path: str | None = None, engine_cls=None, renderer=None,
        reference: dict | None = None, prerender: bool = True, time_boot: bool = True,
        groups: int | None = None) -> dict | None:
    """Run the plan; rank 0 returns the report (None on other ranks).

    ``engine_cls`` / ``renderer`` default to engine.Engine and synth.Renderer (tests pass
    stand-ins to exercise the cross-rank bookkeeping on CPU); ``reference`` maps a global
    shard index to the reference CPU trajectory of that shard (positions [n, 3]).  With
    ``prerender`` the rank's frames are rendered into device memory before the clock starts;
    ``wall`` then covers bootstrap + every step (one host sync at the end, plus one after the
    bootstrap when ``time_boot``).

    ``groups``: the rank's chains are split into this many engines, each on its own HIP
    stream, so that one group's latency-bound stages (PnP, GFTT selection: a block per chain)
    run while another group's tracking fills the GPU (default: ``default_groups(B)``)."""
    dev = torch.device(device or "cuda")
    import torch.distributed as dist
    # world > 1 without a process group: this process runs rank `rank`'s slice of the world-size
    # plan alone (one GPU standing in for one rank of an N-GPU job); the report
    # then covers that slice, and its wall is what that rank would take
    sliced = world > 1 and not (dist.is_available() and dist.is_initialized())
    if engine_cls is None:
        from .engine import Engine as engine_cls
    if renderer is None:
        from .synth import Renderer
        renderer = Renderer(preset, seed=seed, device=dev)
    from .synth import poses
    opts, (b0, b1), _ = Op.get(preset)
    gap = b1 - b0
    plan = Sh.plan_shards(n_frames, world * shards_per_rank, gap, overlap)
    mine = Sh.rank_shards(plan, rank, world)
    B = len(mine)
    Rs, cs = poses(n_frames, renderer.p)
    max_f = max(s.end - s.boot1 + 1 for s in plan)
    G = max(1, min(B, default_groups(B) if groups is None else int(groups)))
    bounds = [(g * B) // G for g in range(G + 1)]
    cuda = dev.type == "cuda"
    engines = [engine_cls(renderer.K, opts, renderer.W, renderer.H, batch=bounds[g + 1] - bounds[g], device=dev,
                          ncap=16384, pcap=16384, fcap=max_f + 8) for g in range(G)]
    # every group on a normal-priority stream of its own.  VO_SEQ_PRIO=1 puts group 0 on a
    # high-priority stream (its bootstrap finishes first and its steps run while the later
    # groups' SIFT fills the GPU): that helped with a device sync after the bootstraps, and costs
    # ~12 % without one (64 shards: 26.1-26.4k vs 29.9k frames/s, profiles/r4_seq_prio.txt)
    prio = os.environ.get("VO_SEQ_PRIO", "0") == "1"
    streams = [torch.cuda.Stream(dev, priority=-1 if (prio and g == 0) else 0) if cuda and G > 1 else None
               for g in range(G)]
    # VO_TRACK_CU_RESERVE=R[:stride] (measurement option): every group's tracking on one stream
    # kept off R compute units (vo_stream_create_cumask), which stay free for the one-block-per-
    # chain PnP / feature-adding / GFTT-selection blocks of the other group
    cu_res = os.environ.get("VO_TRACK_CU_RESERVE", "")
    if cuda and G > 1 and cu_res:
        from . import _lib as L
        r, _, stride = cu_res.partition(":")
        h = C.c_void_p()
        L.check(L.lib().vo_stream_create_cumask(int(r), int(stride or 16), C.byref(h)), "vo_stream_create_cumask")
        ts = torch.cuda.ExternalStream(h.value, device=dev)
        for e in engines:
            e.track_stream = ts

    n_steps = max(s.n_steps for s in mine)
    lo = min(s.start for s in mine)
    hi = min(n_frames, max(s.end for s in mine))
    # frame of chain b at step j: its own next frame, or its last one again once its shard has
    # ended (what the padded chain does then does not count, see final_status below)
    idx = np.array([[min(s.boot1 + 1 + j, s.end - 1, n_frames - 1) for s in mine] for j in range(n_steps)],
                   np.int64).reshape(n_steps, B)
    cache = idx_dev = None
    if prerender:
        # every frame of this rank's shards rendered into HBM before the clock starts (the
        # workload is the VO, not the renderer); ~0.47 MB per KITTI frame.  The per-step frame
        # indices go to the device once too: no host-to-device copy (and so no implicit
        # synchronisation) inside the stepping loop
        cache = torch.empty((hi - lo, renderer.H, renderer.W), dtype=torch.uint8, device=dev)
        for a in range(lo, hi, 32):
            b = min(hi, a + 32)
            cache[a - lo:b - lo] = renderer.render_batch(list(range(a, b)), Rs[a:b], cs[a:b])
        idx_dev = torch.from_numpy(idx - lo).to(dev)
        # every step's frames laid out once as [n_steps][B] (rows of a group contiguous), so a
        # step reads its frames in place: no gather kernel on the critical path of each step
        # (~40 us per group-step at 32 KITTI chains); ~0.47 MB per chain-step
        steps = torch.empty((n_steps, B, renderer.H, renderer.W), dtype=torch.uint8, device=dev)
        for j in range(n_steps):
            torch.index_select(cache, 0, idx_dev[j], out=steps[j])

    def frames_at(ids):
        ids = [min(int(i), n_frames - 1) for i in ids]
        if cache is not None:
            return cache[torch.as_tensor([i - lo for i in ids], device=dev)]
        return renderer.render_batch(ids, Rs[ids], cs[ids])

    boot0 = frames_at([s.start for s in mine])
    boot1 = frames_at([s.boot1 for s in mine])
    # the per-step layout and the two bootstrap frame sets hold every frame the run reads: the
    # rank's frame cache is not needed any more (it doubled the frames' HBM)
    if idx_dev is not None:
        cache = None

    def step_frames(j, g):
        if idx_dev is not None:
            return steps[j, bounds[g]:bounds[g + 1]]
        return frames_at(idx[j, bounds[g]:bounds[g + 1]])

    def on(g):
        return torch.cuda.stream(streams[g]) if streams[g] is not None else _nullctx()

    last = np.array([s.n_steps - 1 for s in mine])
    last_dev = [torch.as_tensor(last[bounds[g]:bounds[g + 1]], device=dev) for g in range(G)]
    # the SIFT workspace is allocated before the clock, as the reference creates its SIFT in
    # the constructor (VisualOdometryPipeLine.py:35) and bench.py's headline reserves it
    for g, eng in enumerate(engines):
        if hasattr(eng, "reserve_bootstrap"):
            with on(g):
                eng.reserve_bootstrap()
    _sync(dev)
    if dist.is_available() and dist.is_initialized():
        dist.barrier()                     # every rank starts its clock together (max-over-ranks wall)
    # without time_boot the groups are not synchronised after their bootstraps (a group steps
    # as soon as its own bootstrap is done); the bootstrap time is then the latest group's
    # end-of-bootstrap event
    ev0 = ev_boot = None
    if not time_boot and cuda:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev0.record(torch.cuda.current_stream(dev))
    t0 = time.perf_counter()
    if G > 1 and cuda:
        for st in streams:
            st.wait_stream(torch.cuda.current_stream(dev))
    for g, eng in enumerate(engines):
        with on(g):
            eng.bootstrap(boot0[bounds[g]:bounds[g + 1]], boot1[bounds[g]:bounds[g + 1]])
            if ev0 is not None:
                if ev_boot is None:
                    ev_boot = []
                e = torch.cuda.Event(enable_timing=True)
                e.record(torch.cuda.current_stream(dev))
                ev_boot.append(e)
    if time_boot:
        _sync(dev)
    t_boot = time.perf_counter() - t0
    # status of every chain at its shard's own last step (chains whose shard has ended keep
    # re-reading their last frame until the longest shard is done; what happens to them then
    # does not count; a shard with no step keeps its bootstrap status, the clone below).
    # Kept on the device, and updated only at the steps where some shard ends.
    final_status = []
    for g, eng in enumerate(engines):
        with on(g):
            final_status.append(eng.t["status"].clone())
    ends = {}
    for g in range(G):
        for j in set(int(v) for v in last[bounds[g]:bounds[g + 1]] if v >= 0):
            ends.setdefault(j, []).append(g)
    for j in range(n_steps):
        for g, eng in enumerate(engines):
            with on(g):
                # with the frames laid out in HBM, the next step's pyramid is built during this
                # step (Engine.step next_frames): tracking then starts each step
                if cuda and idx_dev is not None and j + 1 < n_steps:
                    eng.step(step_frames(j, g), next_frames=step_frames(j + 1, g))
                else:
                    eng.step(step_frames(j, g))
                if g in ends.get(j, ()):
                    final_status[g] = torch.where(last_dev[g] == j, eng.t["status"], final_status[g])
    if G > 1 and cuda:
        for st in streams:
            torch.cuda.current_stream(dev).wait_stream(st)
    host_s = time.perf_counter() - t0
    _sync(dev)
    wall = time.perf_counter() - t0
    if ev_boot:
        t_boot = max(ev0.elapsed_time(e) for e in ev_boot) / 1e3
    t_step = wall - t_boot
    final_status = torch.cat(final_status)
    for eng in engines:
        if hasattr(eng, "release_bootstrap"):
            eng.release_bootstrap()
    t_g = time.perf_counter()
    packed = torch.cat([Sh.pack_poses(e.t["pose_R"], e.t["pose_t"], e.t["nF"], e.dims.fcap) for e in engines])
    allp = Sh.gather_poses(packed)
    if dist.is_available() and dist.is_initialized():
        st_all = [torch.empty_like(final_status) for _ in range(world)]
        dist.all_gather(st_all, final_status.contiguous())
        statuses = torch.cat(st_all).cpu().numpy()
        t_gather = time.perf_counter() - t_g
        tt = torch.tensor([t_step, wall, t_boot, t_gather], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_step, wall, t_boot, t_gather = (float(v) for v in tt.cpu())
    else:
        statuses = final_status.cpu().numpy()
        t_gather = time.perf_counter() - t_g
    if allp is None:
        return None
    t_s = time.perf_counter()
    if sliced:
        plan = mine
    allp = allp.cpu().numpy()
    centres = [Sh.unpack_centres(chain)[: s.end - s.boot1 + 1] for s, chain in zip(plan, allp)]
    ok_shards, ok_centres, failed = [], [], []
    for s, c, st in zip(plan, centres, statuses):
        if st == 0 and len(c) == s.end - s.boot1 + 1:
            ok_shards.append(s)
            ok_centres.append(c)
        else:
            failed.append({"shard": s.index, "status": int(st), "poses": int(len(c))})
    stitched = Sh.stitch(ok_shards, ok_centres) if ok_shards else None
    t_stitch = time.perf_counter() - t_s
    rep = Ev.shard_report(ok_shards, ok_centres, cs, stitched, reference=reference)
    frames_done = sum(s.n_steps for s in plan)
    per = rep["shards"]
    out = {
        "preset": preset, "frames": n_frames, "shards": len(plan), "gpus": world, "chains_per_gpu": shards_per_rank,
        "slice_of_rank": rank if sliced else None,
        "overlap": overlap, "shards_ok": len(ok_shards), "failed_shards": failed,
        "shard_status": {str(int(k)): int(v) for k, v in zip(*np.unique(statuses, return_counts=True))},
        "sequence_frames_per_s": round(n_frames / max(wall, 1e-9), 1),
        "step_frames_per_s": round(frames_done / max(t_step, 1e-9), 1),
        "wall_s": round(wall, 4), "bootstrap_s": round(t_boot, 4), "step_s": round(t_step, 4),
        "steps": n_steps, "groups": G, "host_launch_s": round(host_s, 4),
        # after the clock: pose gather (the collective) and the Sim(3) stitch on rank 0
        "gather_ms": round(t_gather * 1e3, 3), "stitch_ms": round(t_stitch * 1e3, 3),
        "job_frames_per_s": round(n_frames / max(wall + t_gather + t_stitch, 1e-9), 1),
        "shard_ate_rel_max": max((p["ate_rel"] for p in per), default=None),
        "stitched": rep.get("stitched"),
    }
    if reference is not None:
        vs = [p for p in per if "ref_frames" in p]
        out["vs_reference"] = {
            "shards_compared": len(vs),
            "shards_identical": int(sum(p["identical_to_ref"] for p in vs)),
            "ate_rel_max": max((p.get("ate_vs_ref_rel", 0.0) for p in vs), default=None),
        }
    if out_path and stitched is not None:
        keep = ~np.isnan(stitched.positions[:, 0])
        np.savetxt(out_path, np.c_[np.nonzero(keep)[0], stitched.segment[keep], stitched.positions[keep]],
                   fmt=["%d", "%d", "%.9f", "%.9f", "%.9f"])
    out["_stitched"] = stitched
    out["_centres"] = centres
    out["_plan"] = plan
    out["_statuses"] = statuses
    return out


def shard_fixture_paths(golden_dir: str, overlap: int = 30) -> list:
    """The shard fixture files that hold cuts with this overlap (make_long_golden.py): 30 frames
    in kitti_seq00_shards.npz (8, 16) and kitti_seq00_shards_wide.npz (32 .. 256); other overlaps
    in kitti_seq00_shards_o{overlap}.npz."""
    names = ("kitti_seq00_shards.npz", "kitti_seq00_shards_wide.npz") if overlap == 30 else \
        (f"kitti_seq00_shards_o{overlap}.npz",)
    out = []
    for n in names:
        p = os.path.join(golden_dir, n)
        if os.path.exists(p) and int(np.load(p, allow_pickle=False)["overlap"]) == overlap:
            out.append(p)
    return out


def reference_for(golden_dir: str, n_shards: int, overlap: int = 30) -> dict | None:
    """Per-shard reference trajectories of the cut (n_shards, overlap), or None."""
    for p in shard_fixture_paths(golden_dir, overlap):
        r = reference_shards(p, n_shards)
        if r is not None:
            return r
    return None


def reference_shards(path: str, n_shards: int) -> dict | None:
    """Per-shard reference CPU trajectories from tests/golden/kitti_seq00_shards.npz
    (generated by the reference class on the same shard boundaries, make_long_golden.py)."""
    if not os.path.exists(path):
        return None
    g = np.load(path, allow_pickle=False)
    key = f"s{n_shards}_t"
    if key not in g.files:
        return None
    t, off = g[key], g[f"s{n_shards}_off"]
    # the fixture holds transforms[1:] (the bootstrap pose onwards); transforms[0] is the
    # identity at the first bootstrap frame, as in the engine's pose list
    return {k: np.concatenate([np.zeros((1, 3)), t[off[k]:off[k + 1]]]) for k in range(n_shards)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="kitti")
    ap.add_argument("--frames", type=int, default=600)
    ap.add_argument("--shards-per-gpu", type=int, default=8)
    ap.add_argument("--overlap", type=int, default=15)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--reference", default=None, help="per-shard reference trajectories (.npz)")
    ap.add_argument("--out", default=None, help="write the stitched positions (frame segment x y z)")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    ref = reference_shards(args.reference, world * args.shards_per_gpu) if args.reference else None
    res = run(args.preset, args.frames, args.shards_per_gpu, args.overlap, args.seed, dev, rank, world, args.out,
              reference=ref)
    if res is not None:
        print(json.dumps({k: v for k, v in res.items() if not k.startswith("_")}))
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
