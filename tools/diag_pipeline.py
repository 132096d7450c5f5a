"""Diagnostic (not collected by pytest): run the GPU drop-in pipeline on a golden case and
dump per-frame poses/counts next to the fixture's, to gpurun_out/diag_<case>.npz."""
import os
import sys
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), 'tests'))
sys.path.insert(0, os.path.dirname(HERE))
from conftest import golden_frames, load_golden  # noqa: E402
from monocular_visual_odometry_va4mr_amd import options as Op  # noqa: E402
from monocular_visual_odometry_va4mr_amd.VisualOdometryPipeLine import VisualOdometryPipeLine  # noqa: E402
from monocular_visual_odometry_va4mr_amd.ate import ate  # noqa: E402

for case in sys.argv[1:]:
    g = load_golden(case)
    fr = golden_frames(g)
    opts, boot, _ = Op.get(str(g["preset"]))
    vo = VisualOdometryPipeLine(g["K"], opts, max_frames=256, landmark_capacity=4096, candidate_capacity=8192)
    vo.initialization(fr[boot[0]], fr[boot[1]])
    rows = [(len(vo.matched_landmarks), len(vo.potential_keys), vo.num_pts[-1])]
    for i in g["frame"][1:]:
        vo.continuous_operation(fr[i])
        rows.append((len(vo.matched_landmarks), len(vo.potential_keys), vo.num_pts[-1]))
    est = np.array([t.ravel() for _, t in vo.transforms[1:]])
    R = np.array([R for R, _ in vo.transforms[1:]])
    rmse, rel = ate(est, g["t"][:, :, 0])
    os.makedirs("gpurun_out", exist_ok=True)
    np.savez(f"gpurun_out/diag_{case}.npz", t=est, R=R, rows=np.array(rows))
    print(case, "ATE", rmse, rel)
