"""k_sift_retain_best (the SIFT_create(nfeatures) cap, BASELINE C5) on given response arrays,
through the vo_sift_retain_best_rows test hook: the block-parallel partition
rounds must leave the kept keypoints in exactly libstdc++'s std::nth_element /
std::partition order -- pinned against the C oracle (itself pinned against g++'s
std::nth_element in test_retain_best.py) on random, tied, boundary-tied, sorted, organ-pipe
and McIlroy-adversary inputs (the last reaches the depth-limit __heap_select path)."""
import ctypes as C

import numpy as np
import pytest

from test_retain_best import _cases, std_select  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _gpu_retain_best(resp, n_points):
    from monocular_visual_odometry_va4mr_amd import _lib as L
    n = len(resp)
    dev = torch.device("cuda")
    rows = torch.zeros((max(n, 1), 6), dtype=torch.float32)
    rows[:n, 0] = torch.arange(n, dtype=torch.float32)           # original index (exact < 2^24)
    rows[:n, 4] = torch.from_numpy(np.asarray(resp, np.float32))
    rows = rows.to(dev)
    cnt = torch.zeros(8, dtype=torch.int32, device=dev)
    cnt[2] = n
    scratch = torch.zeros(4 * n + 8, dtype=torch.int32, device=dev)
    tmp = torch.zeros(6 * n + 8, dtype=torch.float32, device=dev)
    rc = L.lib().vo_sift_retain_best_rows(C.c_void_p(rows.data_ptr()), n, int(n_points), C.c_void_p(cnt.data_ptr()),
                                          C.c_void_p(scratch.data_ptr()), C.c_void_p(tmp.data_ptr()),
                                          C.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0
    torch.cuda.synchronize()
    kept = int(cnt[2])
    r = rows.cpu().numpy()
    return r[:kept, 0].astype(np.int32), kept, r[:kept, 4]


@pytest.mark.parametrize("name,resp,n_points", list(_cases()), ids=[c[0] for c in _cases()])
def test_gpu_retain_best_matches_oracle(name, resp, n_points):
    from oracle import _olib as O
    perm_o, kept_o = O.retain_best(resp, n_points)
    perm_g, kept_g, resp_g = _gpu_retain_best(resp, n_points)
    assert kept_g == kept_o
    assert np.array_equal(perm_g, perm_o[:kept_o])
    assert np.array_equal(resp_g, resp[perm_o[:kept_o]])


@pytest.mark.parametrize("n,n_points", [(2000, 700), (20000, 8192)])
def test_gpu_retain_best_heap_select_path(std_select, n, n_points):  # noqa: F811
    from oracle import _olib as O
    resp = std_select.killer(n, n_points)
    perm_std, kept_std = std_select(resp, n_points)
    perm_o, kept_o = O.retain_best(resp, n_points)
    assert kept_o == kept_std and np.array_equal(perm_o, perm_std)
    perm_g, kept_g, _ = _gpu_retain_best(resp, n_points)
    assert kept_g == kept_std and np.array_equal(perm_g, perm_std[:kept_std])
