#!/usr/bin/env python3
"""Brute-force 2-NN matcher throughput (SURVEY.md §8d "BF kNN", BASELINE configs C3 / C5).

    python tools/match_bench.py [--B 32] [--n 8192] [--iters 20]

B problems of n x n SIFT-like descriptors (non-negative, L2 norm ~512, clipped to 255 and
rounded, as cv::SIFT writes them) per launch of vo_bf_knn2_batch.  Reports pairs/s and the
MFMA rate of the whole call (prep + MFMA + merge) and of the k_bf_mfma kernel alone
(2 * n * n * 128 FLOP per problem) against the bf16 dense peak.  Prints one JSON line."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from monocular_visual_odometry_va4mr_amd.features import bf_knn2_batch  # noqa: E402

PEAK_BF16 = 2.5e15      # dense bf16 MFMA, MI355X (MI355X_MICROARCH.md)


def sift_like(rng, B, n):
    v = rng.gamma(0.6, 1.0, (B, n, 128)).astype(np.float64)
    v *= 512.0 / np.linalg.norm(v, axis=2, keepdims=True)
    v = np.minimum(v, 0.2 * 512)                      # cv::SIFT clips at 0.2 * norm, renormalises
    v *= 512.0 / np.maximum(np.linalg.norm(v, axis=2, keepdims=True), 1e-9)
    return np.clip(np.rint(v), 0, 255).astype(np.float32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda")
    rng = np.random.default_rng(7)
    q = torch.from_numpy(sift_like(rng, a.B, a.n)).to(dev)
    t = torch.from_numpy(sift_like(rng, a.B, a.n)).to(dev)
    nq = torch.full((a.B,), a.n, dtype=torch.int32, device=dev)
    nt = torch.full((a.B,), a.n, dtype=torch.int32, device=dev)
    for _ in range(3):
        bf_knn2_batch(q, nq, t, nt)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        bf_knn2_batch(q, nq, t, nt)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    flop = 2.0 * a.n * a.n * 128 * a.B
    out = {"tool": "match_bench", "B": a.B, "n": a.n, "ms_per_call": round(ms, 4),
           "pairs_per_s": round(a.B / (ms * 1e-3), 1), "tflops_call": round(flop / (ms * 1e-3) / 1e12, 2),
           "mfma_frac_call": round(flop / (ms * 1e-3) / PEAK_BF16, 4)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
