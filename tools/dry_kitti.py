"""Diagnostic: the drop-in class over synthetic KITTI frames (tests/test_gpu_dataset.py's dry
run) as a plain script, so a bounds-checked library's device printf output is visible.
usage: dry_kitti.py [n_frames] [graph 0/1] [preset]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from monocular_visual_odometry_va4mr_amd import options as Op  # noqa: E402
from monocular_visual_odometry_va4mr_amd.VisualOdometryPipeLine import VisualOdometryPipeLine  # noqa: E402
from monocular_visual_odometry_va4mr_amd.synth import Renderer, poses  # noqa: E402

last = int(sys.argv[1]) if len(sys.argv) > 1 else 12
use_graph = (sys.argv[2] != "0") if len(sys.argv) > 2 else True
preset = sys.argv[3] if len(sys.argv) > 3 else "kitti"
dev = torch.device("cuda")
options, boot, _ = Op.get(preset)
rend = Renderer(preset, seed=1, device=dev)
Rs, cs = poses(last, rend.p)
fr = lambda i: rend.render_batch([i], Rs[i:i + 1], cs[i:i + 1])[0]
vo = VisualOdometryPipeLine(rend.K, options, max_frames=last + 8, device=dev, use_graph=use_graph)
vo.initialization(fr(boot[0]), fr(boot[1]))
torch.cuda.synchronize()
print("bootstrap ok, landmarks", len(vo.matched_landmarks), flush=True)
for i in range(boot[1] + 1, last):
    vo.continuous_operation(fr(i))
    torch.cuda.synchronize()
    print("frame", i, "landmarks", len(vo.matched_landmarks), "cands", len(vo.potential_keys), flush=True)
print("done", flush=True)
