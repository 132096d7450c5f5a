"""The headline's own shape against the reference: bench.py's 768 chains
in 2 stream groups of 384, both groups bootstrapping concurrently on their own streams (no
synchronisation between the groups), then batched steps.  The chains g = 3k bootstrap on the
frames of shard k of the 256-shard cut, whose reference-class runs are in
tests/golden/kitti_seq00_shards_wide.npz (make_long_golden.py): every such chain must match its
shard pose for pose (t_CW and num_pts of every pose, final landmark / candidate counts)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_headline_shape_matches_reference_shards():
    import bench
    dev = torch.device("cuda")
    n_after = 12
    hl = bench.Headline(dev, "kitti", 1, 768, 2, 0, 1, n_after)
    try:
        hl.bootstrap()
        hl.release()
        for j in range(n_after):
            hl.step(2 + j)
        torch.cuda.synchronize()
        st = hl.statuses()
        rep = hl.vs_reference()
        assert rep is not None
        assert rep["compared"] >= 255
        assert rep["covering_every_pose"] >= 253
        assert rep["identical"] == rep["compared"], rep["differences"]
        assert (st == 0).all(), np.unique(st, return_counts=True)
    finally:
        del hl
        torch.cuda.empty_cache()
