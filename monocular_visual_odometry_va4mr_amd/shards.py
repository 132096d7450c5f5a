"""Subsequence sharding across chains and GPUs.

The reference runs one sequence as one chain (main.py:112-124 bootstrap, :166-175 loop).
Here a sequence is cut into contiguous shards; every shard is an independent chain that
bootstraps at [s, s + gap] (gap = bootstrap_frames[1] - bootstrap_frames[0], main.py:18,
48, 78) and runs continuous_operation on [s + gap + 1, e + overlap).  Shards are spread
over ranks (one process per GPU) and over the batch dimension of each rank's Engine; the
only collective is the final gather of per-shard poses to rank 0, which then chains the
shards together with Sim(3) fits on the overlapping camera centres.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from .ate import umeyama


@dataclass(frozen=True)
class Shard:
    index: int          # global shard id
    start: int          # first bootstrap frame
    boot1: int          # second bootstrap frame
    end: int            # one past the last frame processed (includes the overlap)

    @property
    def n_steps(self) -> int:
        return max(0, self.end - self.boot1 - 1)


def plan_shards(seq_len: int, n_shards: int, gap: int, overlap: int = 30) -> list[Shard]:
    """Contiguous shards of [0, seq_len) with ``overlap`` frames shared by neighbours."""
    if n_shards < 1:
        raise ValueError("n_shards must be >= 1")
    out = []
    for k in range(n_shards):
        s = (k * seq_len) // n_shards
        e = ((k + 1) * seq_len) // n_shards
        end = min(seq_len, e + (overlap if k + 1 < n_shards else 0))
        if end - s < gap + 2:
            raise ValueError(f"shard {k} too short: [{s}, {end}) with bootstrap gap {gap}")
        out.append(Shard(k, s, s + gap, end))
    return out


def rank_shards(shards: list[Shard], rank: int, world: int) -> list[Shard]:
    """Round-robin-free block assignment: rank r owns a contiguous block of shards."""
    n = len(shards)
    lo, hi = (rank * n) // world, ((rank + 1) * n) // world
    return shards[lo:hi]


def pack_poses(pose_R: torch.Tensor, pose_t: torch.Tensor, nF: torch.Tensor, fmax: int) -> torch.Tensor:
    """[B, fmax, 13] f64: 9 rotation + 3 translation + valid flag (per chain, frame)."""
    B = pose_R.shape[0]
    out = torch.zeros((B, fmax, 13), dtype=torch.float64, device=pose_R.device)
    f = min(fmax, pose_R.shape[1])
    out[:, :f, :9] = pose_R[:, :f]
    out[:, :f, 9:12] = pose_t[:, :f]
    idx = torch.arange(f, device=pose_R.device)
    out[:, :f, 12] = (idx[None, :] < nF[:, None].to(idx.device)).to(torch.float64)
    return out


def gather_poses(packed: torch.Tensor, group=None) -> torch.Tensor | None:
    """All ranks contribute [B_r, fmax, 13]; rank 0 receives [sum B_r, fmax, 13].

    One all_gather over the process group (RCCL on GPU tensors, gloo on CPU); ranks must
    use equal B (the bench and the shard runner do)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return packed
    world = dist.get_world_size(group)
    parts = [torch.empty_like(packed) for _ in range(world)]
    dist.all_gather(parts, packed.contiguous(), group=group)
    if dist.get_rank(group) != 0:
        return None
    return torch.cat(parts, 0)


def unpack_centres(packed_chain: np.ndarray) -> np.ndarray:
    """Camera centres transforms[k][1] (t_CW, as logged by main.py:172) of one chain."""
    valid = packed_chain[:, 12] > 0.5
    return packed_chain[valid, 9:12]


@dataclass
class Stitched:
    """Result of ``stitch``.

    positions  [total, 3] camera centres, NaN where no shard covers a frame; every segment
               is expressed in the frame of its own first shard
    segment    [total] segment id per frame (-1: not covered)
    segments   shard indices of each segment, in chaining order
    breaks     (previous shard, next shard, common frames) for every place where chaining
               was impossible (< 3 overlapping frames, e.g. a failed shard in between): the
               next shard starts a new segment instead of being placed at an arbitrary pose
    """
    positions: np.ndarray
    segment: np.ndarray
    segments: list
    breaks: list


def stitch_reference(shards: list[Shard], centres: list[np.ndarray], min_common: int = 3) -> Stitched:
    """Shard-by-shard form of ``stitch`` (kept as its test reference): shard k+1 is mapped
    onto shard k's frame by the Sim(3) that aligns their overlapping camera centres
    (Umeyama), accumulated.

    ``centres[k]`` holds poses for frames [boot0] + [boot1 .. end) of shard k, as in
    transforms (index 0 = identity at the first bootstrap frame).  A shard that shares fewer
    than ``min_common`` frames with the previous surviving shard cannot be placed; it opens
    a new segment and the break is reported (a failed shard is reported, not
    silently stitched)."""
    total = max((s.end for s in shards), default=0)
    out = np.full((total, 3), np.nan)
    seg_of = np.full(total, -1, np.int64)
    segments, breaks = [], []

    def frames_of(s: Shard):
        return np.array([s.start] + list(range(s.boot1, s.end)))

    prev_map = None     # frame -> position in the current segment's frame (previous shard)
    prev_shard = None
    for s, c in zip(shards, centres):
        fr = frames_of(s)[:len(c)]
        c = np.asarray(c, np.float64)[:len(fr)]
        common = [] if prev_map is None else [i for i, f in enumerate(fr) if int(f) in prev_map]
        if prev_map is not None and len(common) >= min_common:
            src = c[common]
            dst = np.array([prev_map[int(fr[i])] for i in common])
            sc, R, t = umeyama(src, dst, True)
            segments[-1].append(s.index)
        else:
            if prev_map is not None:
                breaks.append((prev_shard, s.index, len(common)))
            sc, R, t = 1.0, np.eye(3), np.zeros(3)
            segments.append([s.index])
        g = (sc * (R @ c.T)).T + t
        prev_map = {}
        for f, p in zip(fr, g):
            prev_map[int(f)] = p
            if seg_of[f] < 0:
                out[f] = p
                seg_of[f] = len(segments) - 1
        prev_shard = s.index
    return Stitched(out, seg_of, segments, breaks)


def _batched_umeyama(pair, src, dst, n_pairs):
    """Umeyama Sim(3) (ate.umeyama) for many point sets at once: point i belongs to set
    pair[i]; returns s [P], R [P,3,3], t [P,3] with dst ~ s R src + t per set (sets with < 1
    point give the identity)."""
    cnt = np.bincount(pair, minlength=n_pairs).astype(np.float64)
    inv = 1.0 / np.maximum(cnt, 1.0)
    mu_s = np.stack([np.bincount(pair, src[:, d], n_pairs) for d in range(3)], 1) * inv[:, None]
    mu_d = np.stack([np.bincount(pair, dst[:, d], n_pairs) for d in range(3)], 1) * inv[:, None]
    xs, xd = src - mu_s[pair], dst - mu_d[pair]
    outer = (xd[:, :, None] * xs[:, None, :]).reshape(-1, 9)
    cov = np.stack([np.bincount(pair, outer[:, q], n_pairs) for q in range(9)], 1).reshape(-1, 3, 3) * inv[:, None, None]
    U, D, Vt = np.linalg.svd(cov)
    sg = np.where(np.linalg.det(U) * np.linalg.det(Vt) < 0, -1.0, 1.0)
    Sd = np.ones((n_pairs, 3))
    Sd[:, 2] = sg
    R = U @ (Sd[:, :, None] * Vt)
    var_s = np.bincount(pair, (xs ** 2).sum(1), n_pairs) * inv
    sc = np.where(var_s > 0, (D * Sd).sum(1) / np.where(var_s > 0, var_s, 1.0), 1.0)
    t = mu_d - sc[:, None] * np.einsum("pij,pj->pi", R, mu_s)
    return sc, R, t


def stitch(shards: list[Shard], centres: list[np.ndarray], min_common: int = 3) -> Stitched:
    """Chain per-shard trajectories into one: shard k+1 is mapped onto shard k's frame by
    the Sim(3) that aligns their overlapping camera centres (Umeyama), accumulated.

    ``centres[k]`` holds poses for frames [boot0] + [boot1 .. end) of shard k, as in
    transforms (index 0 = identity at the first bootstrap frame).  A shard that shares fewer
    than ``min_common`` frames with the previous surviving shard cannot be placed; it opens
    a new segment and the break is reported (a failed shard is reported, not
    silently stitched).  Where shards overlap, a frame keeps the earliest shard's position.

    Batched (12.9 ms at 256 shards shard by shard): one Umeyama fit per
    consecutive pair in raw shard coordinates, all pairs at once (batched 3x3 SVD); the
    placement of shard k is the product of the pair fits since its segment's first shard,
    formed by a segmented doubling scan over 4x4 similarity matrices.  Umeyama onto
    g(previous) equals g composed with Umeyama onto the previous shard's raw centres for any
    similarity g, so this is the shard-by-shard chaining (``stitch_reference``) up to
    rounding."""
    S = len(shards)
    total = max((s.end for s in shards), default=0)
    out = np.full((total, 3), np.nan)
    seg_of = np.full(total, -1, np.int64)
    if S == 0:
        return Stitched(out, seg_of, [], [])
    # frames of shard k: [start] + [boot1, boot1 + len - 1), truncated to its pose count
    start = np.array([s.start for s in shards], np.int64)
    boot1 = np.array([s.boot1 for s in shards], np.int64)
    lens = np.array([min(len(c), 1 + max(0, s.end - s.boot1)) for s, c in zip(shards, centres)], np.int64)
    off = np.r_[0, np.cumsum(lens)]
    shard_of = np.repeat(np.arange(S), lens)
    j = np.arange(off[-1]) - off[shard_of]                      # pose index within its shard
    allf = np.where(j == 0, start[shard_of], boot1[shard_of] + j - 1)
    allc = np.concatenate([np.asarray(c, np.float64).reshape(-1, 3)[:n] for c, n in zip(centres, lens)])
    n_pairs = S - 1
    if n_pairs > 0:
        # every pose of shards 1.. whose frame the previous shard also has: that shard's pose
        # index there (its bootstrap frame, or boot1 + i - 1)
        sel = shard_of > 0
        f, kp = allf[sel], shard_of[sel] - 1
        in_run = (f >= boot1[kp]) & (f < boot1[kp] + lens[kp] - 1)
        pj = np.where(f == start[kp], 0, np.where(in_run, f - boot1[kp] + 1, -1))
        keep = (pj >= 0) & (pj < lens[kp])
        pair = kp[keep]
        src = allc[np.flatnonzero(sel)[keep]]
        dst = allc[off[pair] + pj[keep]]
        count = np.bincount(pair, minlength=n_pairs)
        sc, R, t = _batched_umeyama(pair, src, dst, n_pairs)
    else:
        count = np.zeros(0, np.int64)
    # per shard k >= 1: its fit onto shard k - 1, or the start of a new segment
    linked = np.r_[False, count >= min_common]
    H = np.tile(np.eye(4), (S, 1, 1))
    if n_pairs > 0:
        H[1:, :3, :3] = sc[:, None, None] * R
        H[1:, :3, 3] = t
    H[~linked] = np.eye(4)
    seg_id = np.cumsum(~linked) - 1
    seg_start = np.flatnonzero(~linked)[seg_id]
    G = H.copy()
    d = 1
    while d < S:                                        # inclusive segmented prefix product
        k = np.arange(d, S)
        ok = k - d >= seg_start[k]
        kk = k[ok]
        if kk.size:
            G[kk] = G[kk - d] @ G[kk]
        d *= 2
    mapped = np.einsum("nij,nj->ni", G[shard_of, :3, :3], allc) + G[shard_of, :3, 3]
    uf, first = np.unique(allf, return_index=True)      # earliest shard covering each frame
    out[uf] = mapped[first]
    seg_of[uf] = seg_id[shard_of[first]]
    idx = [s.index for s in shards]
    segments = [[idx[k] for k in np.flatnonzero(seg_id == g)] for g in range(int(seg_id[-1]) + 1)]
    breaks = [(idx[k - 1], idx[k], int(count[k - 1])) for k in range(1, S) if not linked[k]]
    return Stitched(out, seg_of, segments, breaks)
