#!/usr/bin/env python3
"""How often does the oracle's integer-exact arithmetic (shared bit for bit by the HIP path)
change a result against restatements of OpenCV's fp32 forms?  (CPU only)

The oracle pipeline runs in its exact mode over a synthetic sequence; at every frame the
frame's goodFeaturesToTrack (VisualOdometryPipeLine.py:256) and the pre-step LK call on the
landmarks + candidates (:281,:287) are recomputed with the fp32 restatements
(oracle/vo_oracle_img.c vo_o_set_fp32_mode) and compared with the exact results.
Usage: python tools/opencv_fp32_sensitivity.py [preset] [frames]   (prints one JSON line)"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oracle import _olib as O  # noqa: E402
from oracle import vo_pipeline_oracle as V  # noqa: E402
from monocular_visual_odometry_va4mr_amd import options as Op  # noqa: E402
from monocular_visual_odometry_va4mr_amd.synth import make_sequence  # noqa: E402


def main():
    preset = sys.argv[1] if len(sys.argv) > 1 else "kitti"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    fr, K, _, _ = make_sequence(preset, n, seed={"kitti": 1, "parking": 0, "malaga": 2}.get(preset, 1))
    opts, (b0, b1), _ = Op.get(preset)
    o = opts
    s = V.new_state(K, opts)
    V.initialize(s, fr[b0], fr[b1])
    rec = {"preset": preset, "frames": 0, "gftt_frames_differing": 0, "gftt_corners": 0, "gftt_corners_moved": 0,
           "gftt_lists_equal_length": 0, "lk_points": 0, "lk_status_differing": 0, "lk_pos_differing": 0,
           "lk_pos_max_abs_diff": 0.0}
    for i in range(b1 + 1, n):
        img = fr[i]
        # GFTT on this frame: exact vs fp32 cornerMinEigenVal
        O.set_fp32_mode(0)
        ge = O.gftt(img, o['feature_max_corners'], o['feature_quality_level'], o['feature_min_dist'], o['feature_block_size'])
        O.set_fp32_mode(1)
        gf = O.gftt(img, o['feature_max_corners'], o['feature_quality_level'], o['feature_min_dist'], o['feature_block_size'])
        rec["gftt_corners"] += len(ge)
        same = len(ge) == len(gf) and np.array_equal(ge, gf)
        rec["gftt_frames_differing"] += int(not same)
        rec["gftt_lists_equal_length"] += int(len(ge) == len(gf))
        se = {tuple(p) for p in np.asarray(ge).reshape(-1, 2)}
        sf = {tuple(p) for p in np.asarray(gf).reshape(-1, 2)}
        rec["gftt_corners_moved"] += len(se ^ sf) // 2
        # LK of the points tracked into this frame: exact vs float sums
        pts = np.concatenate([s.kp.reshape(-1, 2), s.cand.reshape(-1, 2)]).astype(np.float32)
        O.set_fp32_mode(0)
        pe, se_, _ = O.lk(s.prev_img, img, pts, tuple(o['winSize']), o['maxLevel'], o['criteria'])
        O.set_fp32_mode(2)
        pf, sf_, _ = O.lk(s.prev_img, img, pts, tuple(o['winSize']), o['maxLevel'], o['criteria'])
        O.set_fp32_mode(0)
        rec["lk_points"] += len(pts)
        rec["lk_status_differing"] += int((se_ != sf_).sum())
        both = (se_ == 1) & (sf_ == 1)
        d = np.abs(pe[both] - pf[both])
        rec["lk_pos_differing"] += int((d > 0).any(1).sum())
        if d.size:
            rec["lk_pos_max_abs_diff"] = max(rec["lk_pos_max_abs_diff"], float(d.max()))
        V.step(s, img)
        rec["frames"] += 1
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
