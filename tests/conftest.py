import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libvo_hip.so)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def load_golden(name):
    d = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
    return {k: d[k] for k in d.files}


_SEQ_CACHE = {}


def golden_frames(g):
    """Re-render the frames of a golden case and check them against the stored digests."""
    from monocular_visual_odometry_va4mr_amd.synth import make_sequence
    import hashlib
    key = (str(g["preset"]), int(g["seed"]), int(g["n_frames"]))
    if key not in _SEQ_CACHE:
        fr, K, _, _ = make_sequence(key[0], key[2], seed=key[1])
        for i, f in enumerate(fr):
            dig = np.frombuffer(hashlib.sha1(f.tobytes()).digest(), np.uint8)
            assert np.array_equal(dig, g["digests"][i]), f"synthetic frame {i} drifted from the fixture"
        _SEQ_CACHE[key] = fr
    return _SEQ_CACHE[key]


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    return torch.cuda.is_available()


@pytest.fixture
def launch_cus():
    """Set the CU count the C ABI's launch-shape decisions assume (vo_set_launch_cus); 1 puts a
    small batch on the many-chains forms (one block per chain: k_essential<2>, k_recover_pose,
    the one-block k_triangulate, k_pnp_tri<2 waves/EU>).  Restored to the device's own count."""
    from monocular_visual_odometry_va4mr_amd import _lib as L

    def set_(n):
        L.check(L.lib().vo_set_launch_cus(int(n)), "vo_set_launch_cus")

    yield set_
    set_(0)
