import sys, numpy as np
sys.path.insert(0, "/root/repo")
from oracle import _olib as O
from oracle import vo_pipeline_oracle as V
from monocular_visual_odometry_va4mr_amd import options as Op
from monocular_visual_odometry_va4mr_amd.synth import Renderer, intrinsics
import oracle.cv2_oracle as CV
got = []
orig = O.find_essential
def hook(p0, p1, K, *a, **k):
    got.append((np.asarray(p0, np.float32).reshape(-1, 2).copy(), np.asarray(p1, np.float32).reshape(-1, 2).copy()))
    return orig(p0, p1, K, *a, **k)
O.find_essential = hook
opts, (b0, b1), _ = Op.get("kitti")
r = Renderer("kitti", seed=1)
starts = [int(s) for s in sys.argv[1:]] or [0, 700, 1400, 2100]
for s0 in starts:
    Rs, cs = r.gt_poses(s0 + b1 + 1)
    fr = r.render_batch([s0, s0 + b1 - b0], Rs[[s0, s0 + b1 - b0]], cs[[s0, s0 + b1 - b0]]).numpy()
    st = V.new_state(intrinsics("kitti"), opts)
    V.initialize(st, fr[0], fr[1])
    print(s0, got[-1][0].shape, flush=True)
np.savez("/tmp/wk/matches.npz", **{f"p0_{i}": a for i, (a, b) in enumerate(got)}, **{f"p1_{i}": b for i, (a, b) in enumerate(got)})
