"""Concurrent use from several HIP streams (the sequence job's stream groups and the headline's
two engines bootstrap at the same time): calls issued on different streams must not share
device scratch.  Regression test for the matcher scratch, which was one buffer per device."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _problem(rng, B, n, dev):
    q = torch.from_numpy(rng.integers(0, 256, (B, n, 128)).astype(np.float32)).to(dev)
    t = torch.from_numpy(rng.integers(0, 256, (B, n, 128)).astype(np.float32)).to(dev)
    nq = torch.full((B,), n, dtype=torch.int32, device=dev)
    nt = torch.full((B,), n - 7, dtype=torch.int32, device=dev)
    return q, nq, t, nt


def test_bf_knn2_batch_concurrent_streams_match_sequential():
    from monocular_visual_odometry_va4mr_amd.features import bf_knn2_batch
    dev = torch.device("cuda")
    rng = np.random.default_rng(5)
    probs = [_problem(rng, 8, 2048, dev), _problem(rng, 8, 1500, dev)]
    seq = [tuple(x.cpu().numpy() for x in bf_knn2_batch(*p)) for p in probs]
    streams = [torch.cuda.Stream(dev) for _ in probs]
    for rep in range(3):
        outs = [None, None]
        for k in (0, 1):
            streams[k].wait_stream(torch.cuda.current_stream(dev))
        # interleave the two streams' calls so the kernels overlap on the GPU
        for _ in range(4):
            for k, p in enumerate(probs):
                with torch.cuda.stream(streams[k]):
                    outs[k] = bf_knn2_batch(*p)
        torch.cuda.synchronize()
        for k in (0, 1):
            i2, d2 = (x.cpu().numpy() for x in outs[k])
            assert np.array_equal(i2, seq[k][0]) and np.array_equal(d2, seq[k][1]), f"rep {rep} stream {k}"
