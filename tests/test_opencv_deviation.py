"""Trajectory-level bound on the oracle's (and the GPU path's) two deliberate departures from
OpenCV's fp32 arithmetic (CPU only, reads committed fixtures).

tools/opencv_trajectory_bound.py ran the reference class (/root/reference/VisualOdometryPipeLine.py
with the oracle shim as cv2) with the oracle's restatements of OpenCV's fp32 forms switched on
(oracle/vo_oracle_img.c vo_o_set_fp32_mode: 1 = cornerMinEigenVal as fp32 Sobel / double box
sums / fp32 lambda, 2 = LK window sums accumulated in float, 3 = both) and stored every pose
(tests/golden/opencv_fp32_trajectories.npz).  Here each is compared with the integer-mode
golden of the same sequence -- the trajectory the GPU reproduces bit for bit -- by ATE
(Umeyama Sim(3) RMSE / path length), next to north_star's 1 % tolerance:

* GFTT in OpenCV's fp32 form: every pose identical on all three sequences (4533 + 94 + 34),
  including the reference run's own stop on the C2 chain ("Not enough keypoints for PnP" at
  frame 4535: the integer-mode run stops there too).
* LK sums in float: the monocular chain is chaotic -- a 0.05 px change in one tracked point
  flips a RANSAC inlier -- and ends 5.1 % (C2, over the 4533 poses both runs have; the float
  run tracks on to frame 4540) / 5.0 % (Parking, 94) / 2e-6 (Malaga 1024, 34) of the path
  away (profiles/r3_opencv_fp32_trajectory.json).
  A 1 % bound against a real OpenCV run therefore needs OpenCV's own float summation order
  (its SSE lane grouping), which no OpenCV in this image can pin: recorded as unpinned
  (DESIGN.md §3)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

FIX = os.path.join(GOLDEN, "opencv_fp32_trajectories.npz")


def _golden(case):
    g = np.load(os.path.join(GOLDEN, f"{case}.npz"), allow_pickle=False)
    t = g["t"]
    return t.reshape(len(t), 3), str(g["error"])


def _golden_t(case):
    return _golden(case)[0]


@pytest.fixture(scope="module")
def fix():
    if not os.path.exists(FIX):
        pytest.skip("opencv_fp32_trajectories.npz not generated (tools/opencv_trajectory_bound.py)")
    return np.load(FIX, allow_pickle=False)


@pytest.mark.parametrize("case", ["kitti_seq00", "parking_c1", "malaga1024_c3"])
def test_fp32_gftt_changes_no_pose(fix, case):
    """OpenCV's fp32 cornerMinEigenVal vs the oracle's integer-exact lambda: same trajectory."""
    t = fix[f"{case}_m1_t"]
    ref, err = _golden(case)
    assert str(fix[f"{case}_m1_error"]) == err         # the same stop (or none) as the integer run
    assert np.array_equal(t, ref)


@pytest.mark.parametrize("case,bound", [("kitti_seq00", 0.10), ("parking_c1", 0.08), ("malaga1024_c3", 1e-4)])
def test_fp32_lk_sum_order_ate(fix, case, bound):
    """LK window sums in float vs int64-exact: every float run tracks to the end, and the ATE
    over the poses both runs have is the measured chaotic divergence recorded in DESIGN §3 --
    above the 1 % tolerance on the long C2 chain and the Parking run."""
    from monocular_visual_odometry_va4mr_amd.ate import ate
    ref, err = _golden(case)
    for mode in (2, 3):
        t = fix[f"{case}_m{mode}_t"]
        assert str(fix[f"{case}_m{mode}_error"]) == ""
        assert len(t) == len(ref) if err == "" else len(t) > len(ref)
        n = len(ref)
        _, rel = ate(t[:n], ref)
        print(f"{case} mode {mode}: ATE {rel:.3e} of the path length")
        assert 0.0 < rel < bound
