#!/usr/bin/env python3
"""Benchmark of the VO per-frame hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--chains B]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (config C2, "KITTI seq00 1241x376 grayscale, full detect->KLT->PnP-RANSAC per-frame
loop"): a seeded synthetic 1241x376 sequence of KITTI seq00's length (4541 frames, K of
utils.py:22-24, options of main.py:20-44).  The job's N*B chains are contiguous
subsequence shards; chain g bootstraps at frames [s_g, s_g+2] (main.py:18) and then runs
continuous_operation (VisualOdometryPipeLine.py:326-373) on the following frames.  All
frames are rendered into HBM before the timed region.

A "step" = one continuous_operation of every chain on its rank (B frames per GPU).  Timed
region: K steps between barrier + device synchronisation; value = frames of the chains of
all ranks that are still tracking (status 0) after the timed region / max-over-ranks time
(weak scaling: B chains per GPU whatever N is).

Extra JSON fields:
  roofline     -- the dominant stage, timed with HIP events recorded on the engine's
                  stream around its launches inside the timed region; achieved =
                  algorithmic bytes (DESIGN.md "Kernels") / mean stage time
  cpu_baseline -- the CPU restatement (oracle/, OpenCV-4.6 semantics, 1 core) timed per
                  frame on this host over a bounded sample (rank 0, N=1 only)
  cpu_baseline_allcores -- the same restatement on up to 16 chains at once, one process
                  each: the all-cores CPU rate (aggregate frames/s)
  ate_vs_ref   -- ATE of the GPU trajectory vs that CPU run on the same frames
  sequence     -- the whole 4541-frame sequence as world x --seq-chains shards, bootstrap
                  included: frames/s = 4541 / wall, per-shard identity with the reference
                  class's runs on the same shard boundaries, stitched ATE (sequence_leg);
                  seq00_frames_per_s repeats its frames/s at the top level
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from monocular_visual_odometry_va4mr_amd import options as Op          # noqa: E402
from monocular_visual_odometry_va4mr_amd.engine import Engine          # noqa: E402
from monocular_visual_odometry_va4mr_amd.synth import Renderer, poses  # noqa: E402
from monocular_visual_odometry_va4mr_amd import shards as Sh           # noqa: E402
from monocular_visual_odometry_va4mr_amd import evaluation as Ev       # noqa: E402

SEQ_LEN = 4541          # KITTI seq00 frame count
SEQ_OVERLAP = 15        # frames shared by neighbouring shards of the sequence job (--seq-overlap)
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8 TB/s
MFMA_PEAK_TF = 2500.0   # dense bf16 MFMA (no sparsity)
MFMA_PEAK_I8 = 5000.0   # dense int8 MFMA: 32x32x32 in the cycles of bf16 32x32x16 (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--chains", type=int, default=768, help="chains (shards) per GPU")
    ap.add_argument("--groups", type=int, default=2,
                    help="split the chains into this many engines, each on its own HIP stream "
                         "(latency-bound stages of one group overlap the others' kernels)")
    ap.add_argument("--preset", default="kitti")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-frames", type=int, default=100, help="CPU-baseline sample length")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16, help="chains (processes) in the all-cores CPU leg (1: skip)")
    ap.add_argument("--cpu-mt-frames", type=int, default=30, help="steps per chain in the multi-thread CPU leg")
    ap.add_argument("--no-single", action="store_true", help="skip the single-chain latency / CPU leg "
                    "(profiling runs of the batched workload)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="per-launch HBM bytes from a rocprofv3 --pmc pass (see profiles/)")
    ap.add_argument("--stages", action="store_true", help="print per-stage times to stderr")
    ap.add_argument("--no-match", action="store_true", help="skip the C3 / C5 legs (SIFT + BF matcher, C5 step)")
    ap.add_argument("--no-sequence", action="store_true", help="skip the whole-sequence leg")
    ap.add_argument("--seq-chains", type=int, default=None,
                    help="shards per GPU of the whole-sequence job (n_shards = world x this; default "
                         "seq_chains_for(world))")
    ap.add_argument("--seq-groups", type=int, default=None, help="stream groups of the sequence job")
    ap.add_argument("--seq-overlap", type=int, default=SEQ_OVERLAP,
                    help="frames shared by neighbouring shards of the sequence job (reference fixtures: "
                         "tests/golden/kitti_seq00_shards*.npz)")
    ap.add_argument("--no-rank-slices", action="store_true",
                    help="skip the one-rank-of-N sequence slices (rank 0 of world 2 / 4 / 8 on this GPU)")
    # hardware queues: the environment's value (HIP's default 4 on the GPU box); --hw-queues N
    # overrides it for experiments (set before HIP initialises; <= 32)
    ap.add_argument("--hw-queues", type=int, default=0,
                    help="GPU_MAX_HW_QUEUES for this process (0 = the environment's value)")
    return ap.parse_args()


class StagePoses:
    """Ground-truth poses for frames [0, n) computed once (synth.poses integrates from 0)."""

    def __init__(self, n, params):
        self.R, self.c = poses(n, params)


def render_windows(rend, gt, starts, gap, n_after, device, chunk=32):
    """frames[j, b] for chain b: j=0 -> s_b, j=1 -> s_b+gap, j>=2 -> s_b+gap+j-1.
    Shard windows overlap, so every distinct frame is rendered once and then gathered."""
    B = len(starts)
    idx = np.array([[s] + [s + gap + j - 1 for j in range(1, 2 + n_after)] for s in starts]).T  # [2+n_after, B]
    idx[1] = np.array(starts) + gap
    uniq, inv = np.unique(idx, return_inverse=True)
    frames_u = torch.empty((len(uniq), rend.H, rend.W), dtype=torch.uint8, device=device)
    for i in range(0, len(uniq), chunk):
        f = uniq[i:i + chunk]
        frames_u[i:i + len(f)] = rend.render_batch(list(f), gt.R[f], gt.c[f])
    out = frames_u[torch.as_tensor(inv.reshape(idx.shape), device=device)]
    del frames_u
    return out


def klt_bytes(eng, n_pts):
    """5*sum(px) prev pyramid+derivatives + sum(px) next pyramid + 17 B/pt."""
    d = eng.dims
    spx = sum(d.lvl_w[i] * d.lvl_h[i] for i in range(d.nlev))
    return 6.0 * spx * eng.B + 17.0 * n_pts


def pyr_bytes(eng):
    """vo_pyr_build: u8 frame read + every pyramid level written (u8, interior pixels) + the
    int16x2 Scharr derivatives of every level written, per chain."""
    d = eng.dims
    spx = sum(d.lvl_w[i] * d.lvl_h[i] for i in range(d.nlev))
    return float(eng.B * (eng.W * eng.H + spx + 4 * spx))


def gftt_bytes(eng, n_corners):
    return float(eng.B * eng.W * eng.H + 8 * n_corners)


def sift_bytes(sift) -> float:
    """SURVEY.md §8d SIFT algorithmic bytes per image: 2 x 11 x 4 B per scale-space pixel (6
    Gaussians + 5 DoG layers, fp32, each written once and read once) over the octaves."""
    sb = sift.sb
    spx = sum(int(sb.oct_w[o]) * int(sb.oct_h[o]) for o in range(sb.n_oct))
    return 88.0 * spx


def sift_match_leg(device, preset, seed, n_frames, nfeatures=0, iters=2):
    """Detect + describe `n_frames` consecutive synthetic frames in ONE vo_sift_batch launch
    sequence, then match the n_frames - 1 consecutive pairs in ONE vo_bf_knn2_batch launch
    (BFMatcher.knnMatch k=2 on MFMA), each timed with HIP events on the current stream.
    Rooflines: SIFT against HBM (sift_bytes per image), BF against the dense int8 MFMA peak
    (2 * nq * nt * 128 integer ops per pair on the real descriptor counts; the bf16 peak when
    VO_BF_BF16=1 selects the bf16 kernel)."""
    from monocular_visual_odometry_va4mr_amd.features import Sift, bf_knn2_batch
    rend = Renderer(preset, seed=seed, device=device)
    Rs, cs = poses(n_frames, rend.p)
    frames = rend.render_batch(list(range(n_frames)), Rs, cs)
    sift = Sift(rend.W, rend.H, device, batch=n_frames, nfeatures=nfeatures)

    def run():
        kp, desc, n = sift.run_batch(frames)
        e1.record()
        out = bf_knn2_batch(desc[:-1], n[:-1], desc[1:], n[1:])
        return n, out

    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    run()
    torch.cuda.synchronize()
    if sift.overflowed(n_frames):
        raise RuntimeError("SIFT capacity exceeded")
    t_sift = t_bf = 0.0
    for _ in range(iters):
        e0.record()
        n, _ = run()
        e2.record()
        torch.cuda.synchronize()
        t_sift += e0.elapsed_time(e1) / iters
        t_bf += e1.elapsed_time(e2) / iters
    nn = n.to(torch.float64).cpu().numpy()
    pairs = n_frames - 1
    flop = float(2.0 * 128 * (nn[:-1] * nn[1:]).sum())
    tf = flop / (t_bf * 1e-3) / 1e12
    sb = sift_bytes(sift) * n_frames
    gbs = sb / (t_sift * 1e-3) / 1e9
    return {"frames": n_frames, "pairs": pairs, "keypoints_mean": round(float(nn.mean()), 1),
            "sift_ms_per_image": round(t_sift / n_frames, 4), "bf_ms_per_pair": round(t_bf / pairs, 4),
            "pairs_per_s": round(pairs / ((t_sift * pairs / n_frames + t_bf) * 1e-3), 1),
            "sift_roofline": {"bound": "hbm", "kernel": "vo_sift_batch", "achieved": round(gbs, 2),
                              "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 5),
                              "algorithmic_bytes_per_image": sift_bytes(sift)},
            "bf_roofline": bf_roofline(tf, flop)}


def bf_roofline(tops, ops):
    if os.environ.get("VO_BF_BF16") == "1":
        return {"bound": "mfma", "kernel": "vo_bf_knn2_batch (k_bf_mfma, bf16)", "achieved": round(tops, 2),
                "peak": MFMA_PEAK_TF, "unit": "TFLOP/s", "frac": round(tops / MFMA_PEAK_TF, 4),
                "flop_per_launch": ops}
    return {"bound": "mfma", "kernel": "vo_bf_knn2_batch (k_bf_i8, int8)", "achieved": round(tops, 2),
            "peak": MFMA_PEAK_I8, "unit": "TOP/s", "frac": round(tops / MFMA_PEAK_I8, 4),
            "flop_per_launch": ops}


def c3_leg(device, n_pairs=16, iters=2):
    """BASELINE config C3 ("Malaga 1024x768, stresses SIFT + BF-match MFMA path"): n_pairs + 1
    consecutive synthetic 1024x768 frames, SIFT detectAndCompute batched over all of them
    (vo_sift_batch) and one batched 2-NN over the consecutive pairs (vo_bf_knn2_batch).
    pairs/s = one new frame's SIFT + one match per pair."""
    r = sift_match_leg(device, "malaga1024", 2, n_pairs + 1, nfeatures=0, iters=iters)
    r["config"] = (f"C3 malaga1024 synthetic, {n_pairs} consecutive pairs: SIFT batched over "
                   f"{n_pairs + 1} frames + batched BF 2-NN")
    return r


def c5_sift_leg(device, n_pairs=16, iters=2):
    """BASELINE config C5's SIFT half ("SIFT capped at the best 8192 + BF 8192^2"): n_pairs + 1
    consecutive synthetic 1920x1080 frames, SIFT_create(nfeatures=8192) batched over all of
    them, the consecutive 8192 x 8192 pairs matched in one launch."""
    r = sift_match_leg(device, "hd1080", 3, n_pairs + 1, nfeatures=8192, iters=iters)
    r["config"] = (f"C5 hd1080 synthetic, {n_pairs} consecutive pairs: SIFT capped at 8192 batched over "
                   f"{n_pairs + 1} frames + batched BF 8192x8192 2-NN")
    return r


def c5_leg(device, chains=256, steps=6, warmup=2, groups=2):
    """BASELINE config C5: synthetic 1920x1080, GFTT maxCorners 8192 /
    qualityLevel 0.01 / minDistance 5 (~8k corners per frame), KLT on all tracked points;
    `chains` shards of the 10,000-frame sequence as batched engines, in `groups` stream groups
    (as the headline).  Frames/s of the per-frame step and the KLT roofline (algorithmic bytes /
    HIP-event stage time of group 0)."""
    opts, (b0, b1), seq_len = Op.get("hd1080")
    gap = b1 - b0
    rend = Renderer("hd1080", seed=3, device=device)
    n_after = warmup + steps
    gt = StagePoses(seq_len, rend.p)
    window = gap + 1 + n_after
    starts = [min((g * seq_len) // chains, seq_len - window) for g in range(chains)]
    frames = render_windows(rend, gt, starts, gap, n_after, device, chunk=16)
    G = max(1, min(groups, chains))
    bounds = [(g * chains) // G for g in range(G + 1)]
    engines = [Engine(rend.K, opts, rend.W, rend.H, batch=bounds[g + 1] - bounds[g], device=device, ncap=65536,
                      pcap=65536, fcap=n_after + 16) for g in range(G)]
    streams = [torch.cuda.Stream(device) if G > 1 else torch.cuda.current_stream(device) for _ in range(G)]
    for g, e in enumerate(engines):
        with torch.cuda.stream(streams[g]):
            e.bootstrap(frames[0, bounds[g]:bounds[g + 1]], frames[1, bounds[g]:bounds[g + 1]])

    def step_all(j, marks=None):
        for g, e in enumerate(engines):
            with torch.cuda.stream(streams[g]):
                e.step(frames[j, bounds[g]:bounds[g + 1]], marks=marks if g == 0 else None)

    for i in range(warmup):
        step_all(2 + i)
    torch.cuda.synchronize()
    nst = len(Engine.STAGES)
    ev = [[[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(nst)] for _ in range(steps)]
    t0 = time.perf_counter()
    for k in range(steps):
        e = ev[k]
        step_all(2 + warmup + k, marks=lambda i, end, strm, e=e: e[i][int(end)].record(strm))
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    eng = engines[0]
    st_ms = np.zeros(nst)
    for k in range(steps):
        for i in range(nst):
            st_ms[i] += ev[k][i][0].elapsed_time(ev[k][i][1])
    st_ms /= steps
    npts = int((eng.t["nL"].to(torch.int64) + eng.t["nC"].to(torch.int64)).sum())
    track_ms = float(st_ms[list(Engine.STAGES).index("track")])
    gbs = klt_bytes(eng, npts) / (track_ms * 1e-3) / 1e9
    # GFTT is the longest stage at C5: eigen pass (HBM: the level-0 image once) + the per-chain
    # ordered selection of up to 8192 corners (one block per chain: latency-bound)
    gftt_ms = float(st_ms[list(Engine.STAGES).index("gftt")])
    ncor = int(eng.t["nCorners"].to(torch.int64).clamp(min=0).sum())
    gftt_gbs = gftt_bytes(eng, ncor) / (gftt_ms * 1e-3) / 1e9
    statuses = np.concatenate([x.statuses() for x in engines])
    n_ok = int((statuses == 0).sum())
    return {"config": f"C5 hd1080 synthetic 1920x1080, {chains} chains in {G} stream group(s), "
                      "maxCorners 8192 / quality 0.01 / minDist 5",
            "frames_per_s": round(n_ok * steps / el, 1), "ms_per_step": round(el / steps * 1e3, 3),
            "points_per_frame": round(npts / eng.B, 1),
            "corners_per_frame": round(float(eng.t["nCorners"].to(torch.float64).mean()), 1),
            "stages_ms": {n: round(float(m), 4) for n, m in zip(Engine.STAGES, st_ms)},
            "track_roofline": {"bound": "hbm", "achieved": round(gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": round(gbs / HBM_PEAK_GBS, 5)},
            "gftt_roofline": {"bound": "latency (per-chain ordered selection)", "stage_ms": round(gftt_ms, 4),
                              "algorithmic_bytes": gftt_bytes(eng, ncor), "achieved": round(gftt_gbs, 2),
                              "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gftt_gbs / HBM_PEAK_GBS, 5)},
            "chains_ok": n_ok}


def seq_chains_for(world: int) -> int:
    """Shards per GPU of the whole-sequence job.  The wall time is bootstrap(B) + (SEQ_LEN /
    (world B) + overlap - 3) x step(B).  Measured at the 15-frame overlap with
    the row-streaming pyramid, rank 0's slice of each plan run alone on one GPU (median of 3-5
    runs, profiles/r5l_slice_sweep_o15*.jsonl): one GPU 48 -> 0.125 s, 64 -> 0.126 s; two GPUs
    48 -> 0.082 s (64: 0.087, 32: 0.108); four 48 -> 0.060 s (64: 0.067, 32: 0.072); eight 24 ->
    0.041-0.056 s (32: 0.043-0.057, 16: 0.065).  So 48 per GPU up to four GPUs and 24 beyond
    (48, 96, 192, 192 shards on 1, 2, 4, 8 GPUs); reference fixtures hold every one of these cuts."""
    return 48 if world <= 4 else 24


def sequence_leg(device, seed, rank, world, per_gpu=48, groups=None, reps=3, overlap=SEQ_OVERLAP):
    """The whole C2 sequence as one job: SEQ_LEN frames cut into
    world x per_gpu overlapping shards (`overlap` frames shared), per_gpu chains on every rank (the
    shards per GPU are the batch dimension, main.py:166-175's loop split across chains),
    bootstrap included in the clock (frames pre-rendered into HBM), poses gathered to rank 0
    and stitched.  frames/s = SEQ_LEN unique frames / wall.  Every shard's trajectory is
    compared with the reference class's own run on the same boundaries when a fixture holds
    that cut (tests/golden/kitti_seq00_shards*.npz, §8e), plus the stitched ATE against ground
    truth.  Run `reps` times; the median run (by wall) is reported and every run's wall is
    listed (`wall_s_runs`, in run order; the first pays one-time costs).
    Wall-time model: bootstrap(B) + n_steps x step(B), n_steps = ceil(SEQ_LEN /
    shards) + overlap - 3: the overlap caps the job once SEQ_LEN / shards approaches it."""
    from monocular_visual_odometry_va4mr_amd.run_sequence import reference_for, run
    n_shards = world * per_gpu
    ref = reference_for(os.path.join(ROOT, "tests", "golden"), n_shards, overlap)
    rnd = seq_renderer(device, seed)
    runs = []
    for _ in range(reps):
        r = run("kitti", SEQ_LEN, per_gpu, overlap=overlap, seed=seed, device=device, rank=rank, world=world,
                reference=ref, time_boot=False, groups=groups, renderer=rnd)
        if r is not None:
            runs.append(r)
        torch.cuda.empty_cache()
    if not runs:
        return None
    res = sorted(runs, key=lambda r: r["wall_s"])[len(runs) // 2]
    st = res.get("stitched") or {}
    vs = res.get("vs_reference")
    # the stitched job against the reference class run as one chain over the whole sequence
    # (informational; rank 0 holds every shard after the gather)
    one = None
    p1 = os.path.join(ROOT, "tests", "golden", "kitti_seq00.npz")
    if os.path.exists(p1) and res.get("_stitched") is not None:
        g1 = np.load(p1, allow_pickle=False)
        if int(g1["seed"]) == seed and int(g1["n_frames"]) == SEQ_LEN:
            one = Ev.stitched_vs_one_chain(res["_stitched"], g1["t"], int(g1["boot"][1]))
    return {"overlap": overlap, "config": f"C2 whole sequence: {SEQ_LEN} frames as {res['shards']} overlapping shards "
                      f"({per_gpu} per GPU, {res['groups']} stream group(s)) on {world} GPU(s), "
                      "bootstrap + every step timed, poses gathered + Sim(3)-stitched after",
            "frames_per_s": res["sequence_frames_per_s"], "wall_s": res["wall_s"], "reported": f"median of {len(runs)} runs",
            "wall_s_runs": [r["wall_s"] for r in runs], "shards": res["shards"],
            "chains_per_gpu": per_gpu, "groups": res["groups"], "shards_ok": res["shards_ok"],
            "bootstrap_s": res["bootstrap_s"], "step_s": res["step_s"], "steps": res["steps"],
            "ms_per_step": round(res["step_s"] / max(1, res["steps"]) * 1e3, 4),
            "chain_steps_per_s": res["step_frames_per_s"],
            "gather_ms": res["gather_ms"], "stitch_ms": res["stitch_ms"],
            "frames_per_s_incl_gather_stitch": res["job_frames_per_s"],
            "failed_shards": res["failed_shards"], "vs_reference": vs,
            "reference_fixture": vs is not None,
            "stitched_frames": st.get("frames"), "coverage_breaks": st.get("coverage_breaks"),
            "stitched_ate_rel_vs_gt": st.get("ate_rel"),
            "stitched_ate_rel_vs_one_chain": one and one["ate_rel"],
            "stitched_vs_one_chain": one}


def rank_slice_leg(device, seed, worlds=(2, 4, 8), reps=5, overlap=SEQ_OVERLAP):
    """What the ranks of an N-GPU sequence job do, measured on this GPU:
    every rank's slice of the world = N plan (N x seq_chains_for(N) shards of the C2 sequence)
    run alone, one rank after another, bootstrap included, every shard compared with the
    reference class's run on the same boundaries.  Ranks run independently until the final
    gather, so the job's wall is the slowest rank's: the predicted rate is SEQ_LEN / max over
    ranks of the rank's wall (median of `reps` runs per rank, after one untimed run of the plan);
    `..._incl_stitch` adds the batched
    stitch of all N x B shards (timed on the reference cut's own poses) -- the RCCL gather of
    ~0.4 MB is not modelled.  The frames come from one cached render of the sequence."""
    from monocular_visual_odometry_va4mr_amd.run_sequence import reference_for, run
    rnd = seq_renderer(device, seed)
    out = {}
    for world in worlds:
        per_gpu = seq_chains_for(world)
        n_shards = world * per_gpu
        ref = reference_for(os.path.join(ROOT, "tests", "golden"), n_shards, overlap)
        ranks = []
        # one untimed run per plan first: the first run of new launch shapes pays one-time costs
        run("kitti", SEQ_LEN, per_gpu, overlap=overlap, seed=seed, device=device, rank=0, world=world,
            reference=None, time_boot=False, renderer=rnd)
        for rank in range(world):
            runs = []
            for _ in range(reps):
                runs.append(run("kitti", SEQ_LEN, per_gpu, overlap=overlap, seed=seed, device=device, rank=rank,
                                world=world, reference=ref, time_boot=False, renderer=rnd))
                torch.cuda.empty_cache()
            ranks.append((sorted(runs, key=lambda r: r["wall_s"])[len(runs) // 2], runs))
        walls = [res["wall_s"] for res, _ in ranks]
        worst = int(np.argmax(walls))
        res0 = ranks[worst][0]
        stitch_ms = stitch_time_ms(ref, n_shards, overlap) if ref else None
        vss = [res.get("vs_reference") or {} for res, _ in ranks]
        cmp_ = [v.get("shards_compared") for v in vss]
        idt = [v.get("shards_identical") for v in vss]
        out[str(world)] = {
            "shards_total": n_shards, "shards_per_rank": per_gpu, "groups": res0["groups"],
            "per_rank_wall_s": walls, "wall_s_runs": [[r["wall_s"] for r in runs] for _, runs in ranks],
            "slowest_rank": worst, "max_wall_s": walls[worst],
            "bootstrap_s": [res["bootstrap_s"] for res, _ in ranks], "steps": [res["steps"] for res, _ in ranks],
            "ms_per_step": [round(res["step_s"] / max(1, res["steps"]) * 1e3, 4) for res, _ in ranks],
            "predicted_frames_per_s": round(SEQ_LEN / walls[worst], 1),
            "rank0_predicted_frames_per_s": round(SEQ_LEN / walls[0], 1),
            "stitch_ms_all_shards": stitch_ms,
            "predicted_frames_per_s_incl_stitch": (round(SEQ_LEN / (walls[worst] + stitch_ms * 1e-3), 1)
                                                   if stitch_ms is not None else None),
            "shards_ok": int(sum(res["shards_ok"] for res, _ in ranks)),
            "shards_compared": None if None in cmp_ else int(sum(cmp_)),
            "shards_identical": None if None in idt else int(sum(idt))}
    return out


_SEQ_RENDER = {}


def seq_renderer(device, seed):
    """The C2 sequence rendered once into HBM (SEQ_LEN frames, ~2.1 GB) for every sequence run
    of this process (the job's frames are pre-rendered before its clock anyway)."""
    from monocular_visual_odometry_va4mr_amd.synth import CachedRenderer, Renderer
    key = (str(device), int(seed))
    if key not in _SEQ_RENDER:
        _SEQ_RENDER[key] = CachedRenderer(Renderer("kitti", seed=seed, device=device), SEQ_LEN)
    return _SEQ_RENDER[key]


def stitch_time_ms(ref: dict, n_shards: int, overlap: int = 30, iters: int = 5) -> float:
    """Median wall of shards.stitch over the reference cut's own per-shard positions (the
    input rank 0 stitches after the gather, at the job's full shard count)."""
    plan = Sh.plan_shards(SEQ_LEN, n_shards, 2, overlap)
    cs = [ref[k] for k in range(n_shards)]
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        Sh.stitch(plan, cs)
        ts.append((time.perf_counter() - t0) * 1e3)
    return round(float(np.median(ts)), 3)


def cpu_baseline(K, opts, frames_np, gap):
    """CPU restatement (oracle/, 1 thread) on one chain: bootstrap (untimed) then the
    per-frame step; median frame time after 10 warm-up frames."""
    from oracle import vo_pipeline_oracle as V
    s = V.new_state(K, opts)
    V.initialize(s, frames_np[0], frames_np[1])
    ts = []
    t_all = time.perf_counter()
    for i in range(2, len(frames_np)):
        t0 = time.perf_counter_ns()
        V.step(s, frames_np[i])
        ts.append((time.perf_counter_ns() - t0) * 1e-9)
    wall = time.perf_counter() - t_all
    med = float(np.median(ts[10:] if len(ts) > 20 else ts))
    pos = np.array([np.asarray(t, np.float64).ravel() for _, t in s.transforms])
    return med, wall, len(ts), pos


def _cpu_chain_worker(K, opts, frames_np, ready, go, out):
    """One CPU-baseline chain in its own process (bench.cpu_baseline_procs)."""
    from oracle import vo_pipeline_oracle as V
    s = V.new_state(K, opts)
    V.initialize(s, frames_np[0], frames_np[1])
    ready.put(1)
    go.wait()
    t0 = time.monotonic()
    for f in range(2, len(frames_np)):
        V.step(s, frames_np[f])
    out.put((t0, time.monotonic(), len(frames_np) - 2))


def cpu_baseline_procs(K, opts, frames_np, procs):
    """The CPU restatement on `procs` independent chains at once, one process per chain
    (spawned interpreters: no GIL sharing, no GPU state), bootstraps untimed; all chains start
    together and the aggregate frames/s is their frames / (last end - first start)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    ready, out, go = ctx.Queue(), ctx.Queue(), ctx.Event()
    ps = [ctx.Process(target=_cpu_chain_worker, args=(K, opts, frames_np, ready, go, out)) for _ in range(procs)]
    for p in ps:
        p.start()
    for _ in range(procs):
        ready.get(timeout=600)
    go.set()
    res = [out.get(timeout=600) for _ in range(procs)]
    for p in ps:
        p.join(timeout=60)
    t0 = min(r[0] for r in res)
    t1 = max(r[1] for r in res)
    return sum(r[2] for r in res) / (t1 - t0), t1 - t0


def gpu_chain_positions(K, opts, frames_dev, device):
    """One chain through the engine (the drop-in class's mode): positions, final status and
    the per-frame latency of continuous_operation (host sync after every frame)."""
    eng = Engine(K, opts, frames_dev.shape[-1], frames_dev.shape[-2], batch=1, device=device,
                 ncap=16384, pcap=16384, fcap=max(64, frames_dev.shape[0] + 8))
    eng.bootstrap(frames_dev[0:1], frames_dev[1:2])
    torch.cuda.synchronize()
    lat = []
    # per frame exactly what the drop-in class does (VisualOdometryPipeLine.continuous_operation):
    # the step, then the chain's status word into pinned memory and one stream synchronisation
    for i in range(2, frames_dev.shape[0]):
        t0 = time.perf_counter()
        eng.step(frames_dev[i:i + 1])
        eng.status_word()
        lat.append(time.perf_counter() - t0)
    ex = eng.export_chain(0)
    pos = np.array([np.asarray(t).ravel() for _, t in ex["transforms"]])
    med = float(np.median(lat[10:] if len(lat) > 20 else lat))
    # the same chain again with the per-frame step replayed from a hipGraph
    eng2 = Engine(K, opts, frames_dev.shape[-1], frames_dev.shape[-2], batch=1, device=device,
                  ncap=16384, pcap=16384, fcap=max(64, frames_dev.shape[0] + 8))
    eng2.bootstrap(frames_dev[0:1], frames_dev[1:2])
    eng2.capture_step()
    torch.cuda.synchronize()
    lat_g = []
    for i in range(2, frames_dev.shape[0]):
        t0 = time.perf_counter()
        eng2.step_graph(frames_dev[i:i + 1])
        eng2.status_word(in_graph=True)
        lat_g.append(time.perf_counter() - t0)
    pos_g = np.array([np.asarray(t).ravel() for _, t in eng2.export_chain(0)["transforms"]])
    same = pos_g.shape == pos.shape and bool(np.array_equal(pos_g, pos))
    med_g = float(np.median(lat_g[10:] if len(lat_g) > 20 else lat_g))
    return pos, ex["status"], med, med_g, same


SHARD_FIXTURE = os.path.join(ROOT, "tests", "golden", "kitti_seq00_shards_wide.npz")


def headline_starts(n_shards: int, window: int) -> list[int]:
    """Bootstrap frame of every chain of the job: chain g starts at g * SEQ_LEN // n_shards
    (clipped so its window fits the sequence).  With 768 chains, g = 3k starts exactly where
    shard k of the 256-shard cut does (and g = 12k where the 64-shard cut's shard k does)."""
    return [min((g * SEQ_LEN) // n_shards, SEQ_LEN - window) for g in range(n_shards)]


class Headline:
    """The headline workload on one rank: B chains as G engines, each on its own HIP stream,
    frames of every step rendered into HBM ([2 + n_after][B][H][W])."""

    def __init__(self, device, preset, seed, B, G, rank, world, n_after, reserve=True):
        opts, (b0, b1), _ = Op.get(preset)
        self.gap = b1 - b0
        self.rend = Renderer(preset, seed=seed, device=device)
        self.K = self.rend.K
        window = self.gap + 1 + n_after
        self.starts_all = headline_starts(world * B, window)
        self.starts = self.starts_all[rank * B:(rank + 1) * B]
        self.gt = StagePoses(SEQ_LEN, self.rend.p)
        t0 = time.perf_counter()
        self.frames = render_windows(self.rend, self.gt, self.starts, self.gap, n_after, device)
        torch.cuda.synchronize()
        self.render_s = time.perf_counter() - t0
        self.G = G = max(1, min(G, B))
        self.bounds = [(g * B) // G for g in range(G + 1)]
        self.engines, self.streams = [], []
        # VO_SHARED_TRACK=1: the groups' tracking launches on one shared stream (Engine.track_stream);
        # =2: the same with the groups' own streams (pyramid, PnP, feature adding) at high priority
        st_mode = os.environ.get("VO_SHARED_TRACK", "0")
        shared = torch.cuda.Stream(device) if G > 1 and st_mode in ("1", "2") else None
        for g in range(G):
            self.engines.append(Engine(self.K, opts, self.rend.W, self.rend.H, batch=self.bounds[g + 1] - self.bounds[g],
                                       device=device, ncap=16384, pcap=16384, fcap=n_after + 16))
            self.streams.append(torch.cuda.Stream(device, priority=-1 if st_mode == "2" else 0) if G > 1
                                else torch.cuda.current_stream(device))
            self.engines[-1].track_stream = shared
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if reserve:
            # SIFT workspace (the reference's SIFT_create), each on the stream its engine
            # bootstraps on: the workspace's first kernels also bring up that stream (a HIP stream
            # of torch's pool is created at its first use, ~6 ms, which the first bootstrap paid)
            for g, e in enumerate(self.engines):
                with torch.cuda.stream(self.streams[g]):
                    e.reserve_bootstrap()
        torch.cuda.synchronize()
        self.boot_alloc_s = time.perf_counter() - t0

    def bootstrap(self):
        """Every group's bootstrap on its own stream, issued back to back (they overlap)."""
        f, bd = self.frames, self.bounds
        for g, e in enumerate(self.engines):
            with torch.cuda.stream(self.streams[g]):
                e.bootstrap(f[0, bd[g]:bd[g + 1]], f[1, bd[g]:bd[g + 1]])

    def release(self):
        for e in self.engines:
            e.release_bootstrap()                     # 64 GB per engine; the later legs bootstrap their own

    def step(self, j, marks=None, prefetch=False):
        """Step j of every group; prefetch: step j + 1's frames are known (they are in HBM), so
        their pyramid is built during this step (Engine.step next_frames)."""
        f, bd = self.frames, self.bounds
        for g, e in enumerate(self.engines):
            with torch.cuda.stream(self.streams[g]):
                nxt = f[j + 1, bd[g]:bd[g + 1]] if prefetch and j + 1 < f.shape[0] else None
                e.step(f[j, bd[g]:bd[g + 1]], marks=marks if g == 0 else None, next_frames=nxt)

    def statuses(self):
        return np.concatenate([e.statuses() for e in self.engines])

    def vs_reference(self, fixture=SHARD_FIXTURE, n_shards=256, max_diffs=16):
        """This rank's chains against the reference class's runs of the shard cut whose shards
        they coincide with (evaluation.chains_vs_shard_cut); None without the fixture."""
        from monocular_visual_odometry_va4mr_amd.evaluation import chains_vs_shard_cut, load_shard_cut
        cut = load_shard_cut(fixture, n_shards)
        if cut is None:
            return None
        torch.cuda.synchronize()
        cat = lambda k: torch.cat([e.t[k] for e in self.engines]).cpu().numpy()
        return chains_vs_shard_cut(cut, self.starts, self.gap, cat("pose_t"), cat("num_pts"), cat("nF"),
                                   cat("nL"), cat("nC"), cat("status"), max_diffs=max_diffs)


def main():
    args = parse()
    if args.hw_queues:
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, max(1, args.hw_queues)))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a ROCm GPU")
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=device)

    def barrier():
        if dist is not None:
            dist.barrier()

    opts, (b0, b1), _ = Op.get(args.preset)
    gap = b1 - b0
    B, K_steps, W_steps = args.chains, args.steps, args.warmup
    n_after = W_steps + K_steps
    hl = Headline(device, args.preset, args.seed, B, args.groups, rank, world, n_after)
    rend, gt, Kmat = hl.rend, hl.gt, hl.K
    H, Wd = rend.H, rend.W
    render_s, boot_alloc_s = hl.render_s, hl.boot_alloc_s
    G, engines = hl.G, hl.engines
    eng = engines[0]
    t0 = time.perf_counter()
    hl.bootstrap()
    torch.cuda.synchronize()
    boot_s = time.perf_counter() - t0
    hl.release()
    step_all = hl.step

    # every step builds the next step's pyramid while it tracks (the frames are in HBM), except
    # across the clock: the last warm-up step and the last timed step do not, so the timed
    # region builds exactly one pyramid per timed step
    for i in range(W_steps):
        step_all(2 + i, prefetch=i + 1 < W_steps)
    torch.cuda.synchronize()

    nst = len(Engine.STAGES)
    # (start, end) HIP events per stage and step, recorded on the stream each stage runs on
    ev = [[[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(nst)] for _ in range(K_steps)]

    barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for k in range(K_steps):
        e = ev[k]
        step_all(2 + W_steps + k, marks=lambda i, end, strm, e=e: e[i][int(end)].record(strm),
                 prefetch=k + 1 < K_steps)
    host_s = time.perf_counter() - t_start          # launch-side time (no sync inside steps)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t_start

    # chains still tracking (status 0) after the timed region: only their frames count; a
    # chain that fails returns early from every kernel and produces no poses
    statuses = hl.statuses()
    n_ok = int((statuses == 0).sum())
    n_ok_all = n_ok
    # the chains that coincide with shards of the reference's 256-shard cut, pose by pose
    # (VERDICT r4 item 1): after the clock, never part of the timed region
    vs_ref = hl.vs_reference() if args.preset == "kitti" and args.seed == 1 else None
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        ok_t = torch.tensor([n_ok], dtype=torch.int64, device=device)
        dist.all_reduce(ok_t, op=dist.ReduceOp.SUM)
        n_ok_all = int(ok_t.item())
        if vs_ref is not None:
            vt = torch.tensor([vs_ref["compared"], vs_ref["identical"], vs_ref["covering_every_pose"]],
                              dtype=torch.int64, device=device)
            dist.all_reduce(vt, op=dist.ReduceOp.SUM)
            vs_ref.update(compared=int(vt[0]), identical=int(vt[1]), covering_every_pose=int(vt[2]))

    # per-stage HIP-event times (ms) of group 0 (events on its stream), mean over timed steps
    st_ms = np.zeros(nst)
    for k in range(K_steps):
        for i in range(nst):
            st_ms[i] += ev[k][i][0].elapsed_time(ev[k][i][1])
    st_ms /= max(1, K_steps)

    # live point counts of the last step (for the KLT algorithmic bytes)
    npts = int((eng.t["nL"].to(torch.int64) + eng.t["nC"].to(torch.int64)).sum())
    ncor = int(eng.t["nCorners"].to(torch.int64).sum())
    gf_pass = eng.t["gf_n"].to(torch.float64)

    # final pose gather to rank 0 (the one collective of the sharded path, §8e)
    t_g = time.perf_counter()
    packed = torch.cat([Sh.pack_poses(e.t["pose_R"], e.t["pose_t"], e.t["nF"], e.dims.fcap) for e in engines])
    allp = Sh.gather_poses(packed)
    torch.cuda.synchronize()
    gather_ms = (time.perf_counter() - t_g) * 1e3

    seq = None
    if not args.no_sequence:
        try:                          # a secondary measurement never costs the headline line
            seq = sequence_leg(device, args.seed, rank, world, per_gpu=args.seq_chains or seq_chains_for(world),
                               groups=args.seq_groups, overlap=args.seq_overlap)
        except Exception as exc:  # noqa: BLE001
            seq = {"error": f"{type(exc).__name__}: {exc}"}
        if world == 1 and not args.no_rank_slices and "error" not in (seq or {}):
            try:
                seq["rank_slices"] = rank_slice_leg(device, args.seed, overlap=args.seq_overlap)
            except Exception as exc:  # noqa: BLE001
                seq["rank_slices"] = {"error": f"{type(exc).__name__}: {exc}"}

    if rank != 0:
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return

    frames_total = n_ok_all * K_steps          # frames of chains that tracked through the timed region
    value = frames_total / elapsed
    names = list(Engine.STAGES)
    stage = {n: round(float(m), 4) for n, m in zip(names, st_ms)}
    bytes_by = {
        "track": klt_bytes(eng, npts),
        "gftt": gftt_bytes(eng, ncor),
        "pyr_build": pyr_bytes(eng),
    }
    # the roofline row is the dominant kernel of the step: k_lk_w (track) has the largest
    # kernel time per step in profiles/r1f_by_grid.csv (rocprofv3 trace of this workload);
    # stage event spans of the latency-bound gftt select / PnP stretch under the 2-stream overlap
    dom = "track"
    dom_ms = float(st_ms[names.index(dom)])
    achieved = bytes_by[dom] / (dom_ms * 1e-3) / 1e9
    traffic = None
    if os.path.exists(args.traffic):
        try:
            with open(args.traffic) as f:
                tj = json.load(f)
            rec = tj.get(dom)
            if rec and int(rec.get("chains", -1)) == eng.B and int(rec.get("groups", 1)) == G:
                traffic = float(rec["bytes_per_launch"])
        except (OSError, ValueError, KeyError):
            traffic = None
    roof = {"bound": "hbm", "kernel": "vo_" + dom, "group_chains": eng.B, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
            "algorithmic_bytes_per_launch": bytes_by[dom], "mean_ms": round(dom_ms, 4)}

    # k_lk_w is issue bound, VALU and the CU's scalar unit together: achieved VALU wave-instructions/s from the
    # profiled instructions per tracked point (profiles/lk_valu.json, rocprofv3 SQ_INSTS_VALU at
    # the same config) x the points of this run / the live track time, against the CDNA4 issue
    # peak (32-wide SIMDs: a wave64 VALU instruction every 2 cycles per SIMD)
    roof_valu = roof_salu = None
    vj = os.path.join(ROOT, "profiles", "lk_valu.json")
    if os.path.exists(vj):
        try:
            with open(vj) as f:
                vr = json.load(f)
            peak_vi = 256 * 4 * 2.4e9 / 2
            ach_vi = float(vr["valu_per_point"]) * npts / (dom_ms * 1e-3)
            roof_valu = {"bound": "valu", "kernel": "k_lk_w", "achieved": round(ach_vi / 1e9, 2), "peak": peak_vi / 1e9,
                         "unit": "G VALU wave-instr/s", "frac": round(ach_vi / peak_vi, 4),
                         "valu_per_point": round(float(vr["valu_per_point"]), 1), "profile": vr.get("tag")}
            # the kernel's other issue limit (round 6): a CU has ONE scalar unit for its four
            # SIMDs, so SALU instructions retire at most once per cycle per CU (256 x 2.4 GHz)
            if vr.get("salu_insts_per_launch") and vr.get("points_per_launch"):
                sp = float(vr["salu_insts_per_launch"]) / float(vr["points_per_launch"])
                peak_si = 256 * 2.4e9
                ach_si = sp * npts / (dom_ms * 1e-3)
                roof_salu = {"bound": "salu (one scalar unit per CU)", "kernel": "k_lk_w", "achieved": round(ach_si / 1e9, 2),
                             "peak": peak_si / 1e9, "unit": "G SALU instr/s", "frac": round(ach_si / peak_si, 4),
                             "salu_per_point": round(sp, 1), "profile": vr.get("tag")}
        except (OSError, ValueError, KeyError):
            roof_valu = None

    out = {
        "metric": "frames/s + ATE vs ref, KITTI seq00 1241x376 @ 1/2/4/8 MI355X",
        "value": round(value, 2),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": K_steps,
        "warmup": W_steps,
        "ms_per_step": round(elapsed / K_steps * 1e3, 4),
        "host_ms_per_step": round(host_s / K_steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "mixed(u8,i32,f32,f64)",
        "data": "synthetic",
        "config": {"workload": "C2 kitti seq00-length synthetic 1241x376, per-frame continuous_operation",
                   "width": Wd, "height": H, "chains_per_gpu": B, "frames_per_step": world * B,
                   "parallelism": f"shards{world}x{B}", "streams_per_gpu": G, "seq_len": SEQ_LEN,
                   "seed": args.seed},
        "roofline": roof,
        "roofline_valu": roof_valu,
        "roofline_salu": roof_salu,
        "stages_ms": stage,
        "chains_ok": n_ok_all,
        "chains_failed": world * B - n_ok_all,
        "frames_counted": frames_total,
        "chain_status": {str(int(k)): int(v) for k, v in zip(*np.unique(statuses, return_counts=True))},
        "headline_vs_reference": vs_ref,
        "points_last_step": npts,
        "gftt_candidates_mean": round(float(gf_pass.mean()), 1),
        "corners_mean": round(ncor / eng.B, 1),
        "bootstrap_s": round(boot_s, 3),
        "bootstrap_workspace_alloc_s": round(boot_alloc_s, 3),
        "render_s": round(render_s, 2),
        "gather_ms": round(gather_ms, 3),
    }
    if seq is not None:
        out["sequence"] = seq
        # the real job's rate (each of the 4541 frames counted once, bootstrap included) beside
        # the windowed `value` (chain-steps of overlapping windows)
        out["seq00_frames_per_s"] = seq.get("frames_per_s")

    if world == 1 and args.cpu_frames > 2 and not args.no_single:
        sample = render_windows(rend, gt, [0], gap, args.cpu_frames - 2, device)[:, 0]
        pos_gpu, st, lat, lat_g, same = gpu_chain_positions(Kmat, opts, sample, device)
        out["single_chain"] = {"frames_per_s": round(1.0 / lat, 1), "ms_per_frame": round(lat * 1e3, 3),
                               "graph_frames_per_s": round(1.0 / lat_g, 1), "graph_identical": same,
                               "note": "one chain (drop-in VisualOdometryPipeLine mode), host sync per frame"}
        if not args.no_cpu:
            fr_np = sample.cpu().numpy()
            med, wall, n, pos_cpu = cpu_baseline(Kmat, opts, fr_np, gap)
            out["cpu_baseline"] = {"value": round(1.0 / med, 3), "unit": "frames/s", "cores": 1, "kind": "port",
                                   "sample": f"1 chain, {args.preset} frames 0,{gap} bootstrap + {n} steps; "
                                             f"median step after 10 warm-up ({wall:.1f}s total)"}
            try:
                ncpu = len(os.sched_getaffinity(0))
            except AttributeError:
                ncpu = os.cpu_count() or 1
            thr = max(1, min(args.cpu_threads, ncpu))
            if thr > 1:
                nmt = min(len(fr_np), 2 + args.cpu_mt_frames)
                fps_mt, wall_mt = cpu_baseline_procs(Kmat, opts, fr_np[:nmt], thr)
                out["cpu_baseline_allcores"] = {
                    "value": round(fps_mt, 3), "unit": "frames/s", "cores": thr, "kind": "port",
                    "sample": f"{thr} chains at once, one process each (all cores of this GPU's CPU share), "
                              f"{nmt - 2} steps per chain after an untimed bootstrap ({wall_mt:.1f}s)"}
            from monocular_visual_odometry_va4mr_amd.ate import ate
            rmse, rel = ate(pos_gpu, pos_cpu)
            out["ate_vs_ref"] = {"rmse": float(rmse), "rel_path": float(rel), "frames": int(len(pos_cpu)),
                                 "gpu_status": int(st)}
        else:
            out["cpu_baseline"] = None
    else:
        out["cpu_baseline"] = None
    if world == 1 and not args.no_match:
        for key, leg in (("c3_sift_match", c3_leg), ("c5_sift_match", c5_sift_leg), ("c5_hd1080", c5_leg)):
            try:                      # secondary configurations never cost the headline line
                out[key] = leg(device)
                torch.cuda.empty_cache()
            except Exception as exc:  # noqa: BLE001
                out[key] = {"error": f"{type(exc).__name__}: {exc}"}
        # the matcher's MFMA roofline on real descriptors: C5's capped SIFT output
        c5s = out.get("c5_sift_match") or {}
        if "bf_roofline" in c5s:
            out["roofline_matcher"] = dict(c5s["bf_roofline"], config=c5s["config"])
    print(json.dumps(out))
    if args.stages:
        print(json.dumps({"stages_ms": stage, "bytes": bytes_by}), file=sys.stderr)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
