"""Parity diagnostics (GPU box): where exactly does the HIP path differ from the oracle?

Prints, per stage, exact-equality results and the first differences:
  sift   GPU SIFT vs O.sift at 640x480, 1241x376, 1024x768, 1920x1080
  boot   drop-in initialization vs the oracle's (golden cases): every state array
  step   12 engine steps vs V.step from a common imported state: every state array
Usage: python tools/diag_parity.py [sift] [boot] [step]
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def cmp(name, a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    if a.shape != b.shape:
        print(f"    {name}: SHAPE {a.shape} vs {b.shape}")
        return False
    if np.array_equal(a, b):
        print(f"    {name}: equal {a.shape}")
        return True
    bad = np.argwhere(a != b)
    print(f"    {name}: {len(bad)} differing elements of {a.size}; first rows {np.unique(bad[:, 0])[:8]}")
    r = bad[0][0]
    print(f"      gpu {a[r]}\n      ora {b[r]}")
    return False


def diag_sift():
    import torch
    from oracle import _olib as O
    from monocular_visual_odometry_va4mr_amd.features import Sift
    from monocular_visual_odometry_va4mr_amd.synth import make_sequence
    for preset, seed in (("parking", 4), ("kitti", 1), ("malaga1024", 2), ("hd1080", 3)):
        fr, _, _, _ = make_sequence(preset, 1, seed=seed)
        img = torch.from_numpy(np.ascontiguousarray(fr[0])).cuda()
        s = Sift(img.shape[1], img.shape[0], "cuda")
        s.run(img)
        kg, dg = s.result()
        t0 = time.time()
        ko, do = O.sift(fr[0])
        print(f"  sift {preset} {fr[0].shape}: gpu {len(kg)} kp, oracle {len(ko)} kp ({time.time() - t0:.1f}s)")
        if len(kg) == len(ko):
            for c, nm in enumerate(("x", "y", "size", "angle", "response", "octave")):
                cmp(nm, kg[:, c], ko[:, c])
            cmp("desc", dg, do)
        else:
            sg = {tuple(r[:2]) for r in kg}
            so = {tuple(r[:2]) for r in ko}
            print(f"    only gpu: {len(sg - so)}  only oracle: {len(so - sg)}")


def diag_boot():
    from conftest import golden_frames, load_golden
    from oracle import vo_pipeline_oracle as V
    from monocular_visual_odometry_va4mr_amd import options as Op
    from monocular_visual_odometry_va4mr_amd.VisualOdometryPipeLine import VisualOdometryPipeLine
    for case in ("kitti_c2", "parking_c1", "malaga_c3"):
        g = load_golden(case)
        fr = golden_frames(g)
        opts, boot, _ = Op.get(str(g["preset"]))
        s = V.new_state(g["K"], opts)
        V.initialize(s, fr[boot[0]], fr[boot[1]])
        vo = VisualOdometryPipeLine(g["K"], opts, max_frames=256, landmark_capacity=4096,
                                    candidate_capacity=8192, use_graph=False)
        vo.initialization(fr[boot[0]], fr[boot[1]])
        print(f"  boot {case}: num_pts gpu {vo.num_pts} oracle {s.num_pts}")
        R_g, t_g = vo.transforms[-1]
        R_o, t_o = s.transforms[-1]
        print(f"    |dR| {np.abs(R_g - R_o).max():.3e} |dt| {np.abs(t_g - t_o).max():.3e}")
        cmp("landmarks", vo.matched_landmarks, s.lm)
        cmp("keypoints", vo.matched_keypoints, s.kp)
        cmp("cand", vo.potential_keys, s.cand)
        cmp("cand_first", vo.potential_first_keys, s.cand_first)
        cmp("cand_tau", vo.potential_transforms, s.cand_tau)
        cmp("inliers", vo.inlier_pts_current, s.inl_pts)


def diag_step(steps=12):
    from conftest import golden_frames, load_golden
    from oracle import vo_pipeline_oracle as V
    from monocular_visual_odometry_va4mr_amd import options as Op
    from monocular_visual_odometry_va4mr_amd.engine import Engine
    for case in ("kitti_c2", "parking_c1", "malaga_c3"):
        g = load_golden(case)
        fr = golden_frames(g)
        opts, boot, _ = Op.get(str(g["preset"]))
        s = V.new_state(g["K"], opts)
        V.initialize(s, fr[boot[0]], fr[boot[1]])
        H, W = fr[0].shape
        eng = Engine(g["K"], opts, W, H, batch=1, ncap=4096, pcap=8192, fcap=256)
        eng.import_chain(0, landmarks=s.lm, keypoints=s.kp, cand=s.cand, cand_first=s.cand_first,
                         cand_tau=s.cand_tau, transforms=s.transforms, num_pts=s.num_pts, prev_img=s.prev_img)
        for k in range(min(steps, len(fr) - boot[1] - 1)):
            i = boot[1] + 1 + k
            V.step(s, fr[i])
            eng.step(fr[i])
            e = eng.export_chain(0)
            R_o, t_o = s.transforms[-1]
            R_g, t_g = e["transforms"][-1]
            ok = all([np.array_equal(e["landmarks"], s.lm), np.array_equal(e["keypoints"], s.kp),
                      np.array_equal(e["cand"], s.cand), np.array_equal(e["cand_first"], s.cand_first),
                      np.array_equal(e["cand_tau"], s.cand_tau), np.array_equal(R_g, R_o), np.array_equal(t_g, t_o)])
            print(f"  step {case} frame {i}: status {e['status']} exact={ok} N {len(e['landmarks'])}/{len(s.lm)} "
                  f"P {len(e['cand'])}/{len(s.cand)} |dR| {np.abs(R_g - R_o).max():.2e} |dt| {np.abs(t_g - t_o).max():.2e}")
            if not ok:
                cmp("landmarks", e["landmarks"], s.lm)
                cmp("keypoints", e["keypoints"], s.kp)
                cmp("cand", e["cand"], s.cand)
                cmp("cand_first", e["cand_first"], s.cand_first)
                cmp("cand_tau", e["cand_tau"], s.cand_tau)
                # re-sync so later frames test one step each
                eng.import_chain(0, landmarks=s.lm, keypoints=s.kp, cand=s.cand, cand_first=s.cand_first,
                                 cand_tau=s.cand_tau, transforms=s.transforms, num_pts=s.num_pts,
                                 prev_img=s.prev_img)


if __name__ == "__main__":
    what = sys.argv[1:] or ["sift", "boot", "step"]
    for w in what:
        print(f"== {w}", flush=True)
        {"sift": diag_sift, "boot": diag_boot, "step": diag_step}[w]()
