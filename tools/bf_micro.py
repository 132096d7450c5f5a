"""BF 2-NN alone at BASELINE C5's size (16 problems x 8192 x 8192, SIFT-like integer
descriptors), for kernel traces / counters: python tools/bf_micro.py [reps]."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from monocular_visual_odometry_va4mr_amd.features import bf_knn2_batch  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda")
g = torch.Generator(device="cpu").manual_seed(3)
B, N = 16, 8192
# SIFT-like: mostly small values, a few large (clipped at 255)
q = torch.clamp(torch.distributions.Gamma(0.7, 0.02).sample((B, N, 128)), 0, 255).floor().to(dev)
t = torch.clamp(torch.distributions.Gamma(0.7, 0.02).sample((B, N, 128)), 0, 255).floor().to(dev)
n = torch.full((B,), N, dtype=torch.int32, device=dev)
bf_knn2_batch(q, n, t, n)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    bf_knn2_batch(q, n, t, n)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
print(f"bf_knn2_batch {B}x{N}x{N}: {ms:.4f} ms/launch, {2.0 * 128 * B * N * N / ms / 1e9:.1f} TOP/s (whole call)")
