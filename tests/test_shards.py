"""Sharded multi-GPU path on the CPU: shard planning, pose packing, the one collective
(all_gather of per-chain poses, gloo world_size 2 here, RCCL on GPUs) and Sim(3)
stitching of overlapping shard trajectories."""
import os
import socket

import numpy as np
import pytest
import torch

from monocular_visual_odometry_va4mr_amd import shards as Sh


def test_plan_shards_cover_sequence_with_overlap():
    sh = Sh.plan_shards(4541, 8, gap=2, overlap=30)
    assert sh[0].start == 0 and sh[-1].end == 4541
    for a, b in zip(sh, sh[1:]):
        assert b.start < a.end                  # overlap
        assert a.end - b.start >= 30 - 1
        assert b.boot1 == b.start + 2
    assert sum(s.n_steps for s in sh) >= 4541 - 8 * 3
    with pytest.raises(ValueError):
        Sh.plan_shards(10, 8, gap=6, overlap=0)


def test_rank_shards_partition():
    sh = Sh.plan_shards(1000, 10, gap=2)
    got = [s.index for r in range(3) for s in Sh.rank_shards(sh, r, 3)]
    assert got == list(range(10))


def _traj(n, seed=0):
    rng = np.random.default_rng(seed)
    steps = np.c_[rng.normal(0, 0.05, n), rng.normal(0, 0.02, n), np.ones(n)]
    return np.cumsum(steps, 0)


def _sim3(p, s, ang, t):
    R = np.array([[np.cos(ang), 0, np.sin(ang)], [0, 1, 0], [-np.sin(ang), 0, np.cos(ang)]])
    return (s * (R @ p.T)).T + t


def test_stitch_recovers_global_trajectory():
    gt = _traj(300)
    sh = Sh.plan_shards(300, 3, gap=2, overlap=30)
    centres = []
    for k, s in enumerate(sh):
        fr = np.array([s.start] + list(range(s.boot1, s.end)))
        # each shard sees its own frame: unknown scale / rotation / origin
        centres.append(_sim3(gt[fr], 0.5 + k, 0.2 * k, np.array([k, -k, 2.0 * k])))
    res = Sh.stitch(sh, centres)
    assert res.breaks == [] and res.segments == [[0, 1, 2]]
    out = res.positions
    # frames strictly between a shard's two bootstrap frames have no pose (as in the
    # reference, main.py:112-124); overlaps cover them for every shard but the first
    missing = np.nonzero(np.isnan(out[:, 0]))[0]
    assert missing.tolist() == [1]
    from monocular_visual_odometry_va4mr_amd.ate import ate
    keep = ~np.isnan(out[:, 0])
    rmse, rel = ate(out[keep], gt[keep])
    assert rel < 1e-9


def test_pack_poses_layout():
    B, F = 3, 6
    R = torch.arange(B * F * 9, dtype=torch.float64).reshape(B, F, 9)
    t = torch.arange(B * F * 3, dtype=torch.float64).reshape(B, F, 3)
    nF = torch.tensor([2, 6, 0], dtype=torch.int32)
    p = Sh.pack_poses(R, t, nF, 8)
    assert p.shape == (B, 8, 13)
    assert torch.equal(p[:, :F, :9], R) and torch.equal(p[:, :F, 9:12], t)
    assert p[0, :, 12].tolist() == [1, 1, 0, 0, 0, 0, 0, 0]
    assert p[2, :, 12].sum() == 0
    c = Sh.unpack_centres(p[1].numpy())
    assert c.shape == (6, 3)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    B, F = 2, 5
    R = torch.full((B, F, 9), float(rank), dtype=torch.float64)
    t = torch.full((B, F, 3), 10.0 + rank, dtype=torch.float64)
    nF = torch.tensor([F, F - rank], dtype=torch.int32)
    out = Sh.gather_poses(Sh.pack_poses(R, t, nF, F))
    if rank == 0:
        q.put(out.numpy())
    else:
        q.put(None)
    dist.barrier()
    dist.destroy_process_group()


def test_gather_poses_gloo_world2():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    out = [r for r in res if r is not None][0]
    assert out.shape == (4, 5, 13)
    assert np.all(out[:2, :, :9] == 0) and np.all(out[2:, :, :9] == 1)
    assert np.all(out[:2, :, 9:12] == 10) and np.all(out[2:, :, 9:12] == 11)
    assert out[3, :, 12].tolist() == [1, 1, 1, 1, 0]


def test_stitch_reports_coverage_break_instead_of_identity():
    """A failed middle shard leaves its neighbours without common frames: the later shard
    must open a new segment (reported as a break), not be placed at an identity Sim(3)."""
    gt = _traj(300)
    sh = Sh.plan_shards(300, 3, gap=2, overlap=30)
    centres = []
    for k, s in enumerate(sh):
        fr = np.array([s.start] + list(range(s.boot1, s.end)))
        centres.append(_sim3(gt[fr], 0.5 + k, 0.2 * k, np.array([k, -k, 2.0 * k])))
    keep = [sh[0], sh[2]]                       # shard 1 failed and was dropped
    res = Sh.stitch(keep, [centres[0], centres[2]])
    assert res.breaks == [(0, 2, 0)]
    assert res.segments == [[0], [2]]
    s2 = sh[2]
    f2 = np.array([s2.start] + list(range(s2.boot1, s2.end)))
    assert (res.segment[f2] == 1).all()
    # the second segment stays in its own frame (identical to shard 2's own centres) ...
    assert np.allclose(res.positions[f2], centres[2])
    # ... and the report evaluates each segment on its own, listing the break
    from monocular_visual_odometry_va4mr_amd import evaluation as E
    rep = E.shard_report(keep, [centres[0], centres[2]], gt, res)
    st = rep["stitched"]
    assert st["coverage_breaks"] == [[0, 2, 0]] and len(st["segments"]) == 2
    assert all(seg["ate_rel"] < 1e-9 for seg in st["segments"])
    assert "ate_rel" not in st


class _StubRenderer:
    """Frame source for run_sequence on CPU: a 'frame' is just its index."""

    def __init__(self):
        from monocular_visual_odometry_va4mr_amd.synth import SceneParams, intrinsics
        self.p, self.K, self.W, self.H = SceneParams(), intrinsics("parking"), 4, 1

    def render_batch(self, ids, R, c):
        return torch.tensor([[float(i)] for i in ids], dtype=torch.float64)


class _StubEngine:
    """Stands in for engine.Engine: each chain appends the true camera centre of the frame it
    is given, in its own Sim(3) frame; the chain of the shard that bootstraps at
    ``fail_start`` fails at its 20th step, and every chain 'fails' when fed the same frame
    twice (the padding after its shard has ended) -- which must not count against it."""

    fail_start = 50

    def __init__(self, K, opts, W, H, batch, device, ncap, pcap, fcap):
        from types import SimpleNamespace
        from monocular_visual_odometry_va4mr_amd.synth import SceneParams, poses
        self.B = batch
        self.dims = SimpleNamespace(fcap=fcap)
        self.gt = poses(400, SceneParams())[1]
        self.t = {"pose_R": torch.zeros(batch, fcap, 9, dtype=torch.float64),
                  "pose_t": torch.zeros(batch, fcap, 3, dtype=torch.float64),
                  "nF": torch.ones(batch, dtype=torch.int32), "status": torch.zeros(batch, dtype=torch.int32)}
        self.rank = int(os.environ.get("RANK", "0"))
        self.last = [-1] * batch
        self.steps = 0

    def _append(self, b, f):
        k = int(self.t["nF"][b])
        sc = 0.5 + 0.01 * self.first[b]
        self.t["pose_t"][b, k] = torch.from_numpy(sc * (self.gt[f] - self.gt[self.first[b]]))
        self.t["pose_R"][b, k] = torch.eye(3, dtype=torch.float64).reshape(9)
        self.t["nF"][b] = k + 1

    def bootstrap(self, f0, f1):
        self.first = [int(v) for v in f0[:, 0]]
        for b in range(self.B):
            self._append(b, int(f1[b, 0]))
            self.last[b] = int(f1[b, 0])

    def step(self, frames):
        self.steps += 1
        for b in range(self.B):
            f = int(frames[b, 0])
            if self.t["status"][b] != 0:
                continue
            if f == self.last[b] or (self.first[b] == self.fail_start and self.steps == 20):
                self.t["status"][b] = 1
                continue
            self._append(b, f)
            self.last[b] = f


def _seq_worker(rank, world, port, q, per_rank=2, groups=None):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["RANK"] = str(rank)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from monocular_visual_odometry_va4mr_amd.run_sequence import run
    _StubEngine.fail_start = Sh.plan_shards(200, world * per_rank, 2, 30)[1].start
    res = run("parking", 200, per_rank, overlap=30, device="cpu", rank=rank, world=world,
              engine_cls=_StubEngine, renderer=_StubRenderer(), prerender=False, groups=groups)
    q.put(None if res is None else {k: v for k, v in res.items() if not k.startswith("_")})
    dist.barrier()
    dist.destroy_process_group()


def test_run_sequence_bookkeeping_gloo_world2():
    """run_sequence across 2 ranks (gloo): statuses are gathered with the poses, the failed
    shard (rank 0, chain 1 = shard 1) is reported and dropped, the shard after it cannot be
    chained and opens a new segment (coverage break), and chains that 'fail' only while
    re-reading their last frame after their shard ended still count as complete."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_seq_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(2)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    rep = [r for r in res if r is not None][0]
    assert rep["shards"] == 4 and rep["shards_ok"] == 3
    assert [f["shard"] for f in rep["failed_shards"]] == [1]
    st = rep["stitched"]
    assert st["coverage_breaks"] == [[0, 2, 0]]
    assert [s["shards"] for s in st["segments"]] == [[0], [2, 3]]
    assert all(s["ate_rel"] < 1e-9 for s in st["segments"])


def test_run_sequence_world_x_bseq_plan_gloo_world2():
    """The sequence job's plan n_shards = world x B_seq (bench.py's sequence leg): 2 ranks x 4
    shards, each rank's 4 chains split into 2 stream groups (engines).  Shard order, the
    per-rank blocks and the groups must line up: shard 1 (rank 0, group 0, chain 1) fails and
    is dropped; shard 2 shares one frame with shard 0 (Parking's bootstrap gap is 6), so it
    opens a new segment (a reported break); the others stitch exactly (every stand-in chain is
    a Sim(3) image of the ground truth)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_seq_worker, args=(r, 2, port, q, 4, 2)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(2)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    rep = [r for r in res if r is not None][0]
    assert rep["shards"] == 8 and rep["chains_per_gpu"] == 4 and rep["groups"] == 2
    assert rep["shards_ok"] == 7 and [f["shard"] for f in rep["failed_shards"]] == [1]
    st = rep["stitched"]
    assert st["coverage_breaks"] == [[0, 2, 1]]
    assert [s["shards"] for s in st["segments"]] == [[0], [2, 3, 4, 5, 6, 7]]
    assert all(s["ate_rel"] < 1e-9 for s in st["segments"])


@pytest.mark.parametrize("n_shards,drop", [(3, []), (8, [3]), (64, [1, 2]), (256, [100]), (256, [])])
def test_batched_stitch_equals_shard_by_shard(n_shards, drop):
    """stitch (batched Umeyama over all consecutive pairs + segmented prefix product) against
    the shard-by-shard chaining it replaces (stitch_reference): same segments, breaks and
    coverage, positions equal up to rounding -- with dropped shards (coverage breaks) and a
    truncated first shard."""
    n = 4541
    gt = _traj(n, seed=3)
    rng = np.random.default_rng(n_shards)
    sh = Sh.plan_shards(n, n_shards, gap=2, overlap=30)
    cs = []
    for k, s in enumerate(sh):
        fr = np.array([s.start] + list(range(s.boot1, s.end)))
        cs.append(_sim3(gt[fr], 0.5 + 0.01 * k, 0.1 * k, np.array([k, -k, 2.0 * k])) + rng.normal(0, 1e-3, (len(fr), 3)))
    keep = [s for i, s in enumerate(sh) if i not in drop]
    kc = [c for i, c in enumerate(cs) if i not in drop]
    kc[0] = kc[0][:-5]
    a, b = Sh.stitch_reference(keep, kc), Sh.stitch(keep, kc)
    assert a.breaks == b.breaks and a.segments == b.segments
    assert np.array_equal(a.segment, b.segment)
    m = ~np.isnan(a.positions[:, 0])
    assert np.array_equal(m, ~np.isnan(b.positions[:, 0]))
    assert np.allclose(a.positions[m], b.positions[m], rtol=0, atol=1e-9 * (1 + np.abs(a.positions[m]).max()))


def test_run_sequence_rank_slice_without_process_group():
    """world > 1 without torch.distributed: the process runs rank r's slice of the world-size
    plan alone (bench.py's rank_slices: one GPU standing in for one rank of an N-GPU job); the
    report covers exactly that slice's shards."""
    from monocular_visual_odometry_va4mr_amd.run_sequence import run
    plan = Sh.plan_shards(200, 3 * 2, 2, 30)
    _StubEngine.fail_start = -1
    for rank in range(3):
        rep = run("parking", 200, 2, overlap=30, device="cpu", rank=rank, world=3, engine_cls=_StubEngine,
                  renderer=_StubRenderer(), prerender=False)
        mine = Sh.rank_shards(plan, rank, 3)
        assert rep["slice_of_rank"] == rank and rep["shards"] == len(mine) == 2
        assert [s.index for s in rep["_plan"]] == [s.index for s in mine]
        assert rep["shards_ok"] == 2 and rep["failed_shards"] == []
        assert rep["stitched"]["coverage_breaks"] == []
