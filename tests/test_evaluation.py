"""Trajectory I/O and evaluation helpers (CPU)."""
import numpy as np

from monocular_visual_odometry_va4mr_amd import evaluation as E
from monocular_visual_odometry_va4mr_amd import shards as Sh
from monocular_visual_odometry_va4mr_amd.synth import SceneParams, poses


def _gt(n):
    Rs, cs = poses(n, SceneParams())
    return np.concatenate([Rs, cs[:, :, None]], 2)


def test_kitti_pose_file_roundtrip(tmp_path):
    P = _gt(20)
    f = tmp_path / "poses.txt"
    E.write_kitti_poses(str(f), [(p[:, :3], p[:, 3:]) for p in P])
    Q = E.read_kitti_poses(str(f))
    assert Q.shape == (20, 3, 4) and np.allclose(P, Q, atol=1e-11)
    # the columns the reference plots (utils.py:19-20): t_x = [-9], t_z = [-1]
    row = np.loadtxt(str(f))[5]
    assert np.isclose(row[-9], P[5, 0, 3]) and np.isclose(row[-1], P[5, 2, 3])


def test_rpe_zero_for_scaled_copy_and_detects_drift():
    P = _gt(60)
    est = P.copy()
    est[:, :, 3] *= 3.0                      # monocular scale ambiguity
    t, r = E.rpe(est, P, delta=5)
    assert t < 1e-9 and r < 1e-6
    bad = est.copy()
    bad[30:, 0, 3] += 2.0                    # a jump
    t2, _ = E.rpe(bad, P, delta=1)
    assert t2 > 0.05


def test_shard_report_on_perfect_shards():
    P = _gt(200)
    gt = P[:, :, 3]
    sh = Sh.plan_shards(200, 2, gap=2, overlap=30)
    centres = []
    for s in sh:
        fr = np.array([s.start] + list(range(s.boot1, s.end)))
        centres.append(gt[fr] * 0.7 + 1.0)
    st = Sh.stitch(sh, centres)
    rep = E.shard_report(sh, centres, gt, st)
    assert all(p["ate_rel"] < 1e-9 for p in rep["shards"])
    assert rep["stitched"]["ate_rel"] < 1e-9 and rep["stitched"]["frames"] == 199
