"""ctypes binding of oracle/_build/libvo_oracle.so (CPU ORACLE, test infrastructure only)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libvo_oracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = C.CDLL(_LIB_PATH)
        _declare(_lib)
    return _lib


P = C.c_void_p
I = C.c_int
D = C.c_double


def _declare(L):
    L.vo_o_gftt.argtypes = [P, I, I, I, D, D, I, I, D, P, I, P]
    L.vo_o_eigmap.argtypes = [P, I, I, I, I, D, P]
    L.vo_o_pyrdown.argtypes = [P, I, I, P]
    L.vo_o_scharr.argtypes = [P, I, I, P]
    L.vo_o_pyr_maxlevel.argtypes = [I, I, I, I, I]
    L.vo_o_lk.argtypes = [P, P, I, I, P, I, P, P, P, I, I, I, I, I, D, D]
    L.vo_o_triangulate.argtypes = [P, P, P, P, I, P]
    L.vo_o_triangulate_d.argtypes = [P, P, P, P, I, P]
    L.vo_o_rodrigues_v2m.argtypes = [P, P]
    L.vo_o_rodrigues_m2v.argtypes = [P, P]
    L.vo_o_pnp_ransac_p3p.argtypes = [P, P, I, P, I, D, D, P, P, P, P, P, P]
    L.vo_o_p3p.argtypes = [P, P, P, P, P]
    L.vo_o_epnp.argtypes = [P, P, P, I, P, P]
    L.vo_o_find_essential.argtypes = [P, P, I, P, D, D, I, P, P, P]
    L.vo_o_five_point.argtypes = [P, P, P]
    L.vo_o_recover_pose.argtypes = [P, P, P, I, P, P, P, P, P]
    L.vo_o_sift.argtypes = [P, I, I, P, P, I, P]
    L.vo_o_sift_n.argtypes = [P, I, I, I, P, P, I, P]
    L.vo_o_retain_best.argtypes = [P, I, I, P]
    L.vo_o_retain_best_heap_selects.argtypes = []
    L.vo_o_bf_knn2.argtypes = [P, I, P, I, I, P, P]
    L.vo_o_set_fp32_mode.argtypes = [I]
    L.vo_o_set_fp32_mode.restype = None
    L.vo_o_set_svd_form.argtypes = [I]
    L.vo_o_set_svd_form.restype = None
    L.vo_o_get_svd_form.argtypes = []
    L.vo_o_get_svd_form.restype = I
    L.vo_o_rng_next.argtypes = [P]
    L.vo_o_rng_next.restype = C.c_uint32


def set_fp32_mode(mode: int) -> None:
    """0: integer-exact GFTT / LK sums (the parity oracle); bit 0: OpenCV-style fp32
    cornerMinEigenVal; bit 1: LK sums in float (measurement only, see vo_oracle_img.c)."""
    lib().vo_o_set_fp32_mode(int(mode))


def set_svd_form(form: int) -> None:
    """EPnP's 12x12 SVD of M^T M: 0 = QUARTER_SUM partial sums + u / wn rotation (the GPU's order;
    every golden fixture assumes it), 1 = the round-2 serial sums + t / c / s rotation (an
    independent cross-check, never the parity oracle)."""
    lib().vo_o_set_svd_form(int(form))


def get_svd_form() -> int:
    return int(lib().vo_o_get_svd_form())


def ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def c_u8(a):
    return np.ascontiguousarray(a, dtype=np.uint8)


def c_f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def c_f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


# ------------------------------------------------------------------ thin wrappers
def gftt(img, max_corners, quality, min_dist, block_size=3, use_harris=False, k=0.04):
    img = c_u8(img)
    h, w = img.shape
    cap = max(int(max_corners), 0) or w * h
    cap = min(cap, w * h)
    out = np.zeros((max(cap, 1), 2), np.float32)
    n = C.c_int(0)
    rc = lib().vo_o_gftt(ptr(img), w, h, int(max_corners), float(quality), float(min_dist),
                         int(block_size), int(bool(use_harris)), float(k), ptr(out), cap, C.byref(n))
    if rc < 0:
        raise RuntimeError(f"vo_o_gftt failed rc={rc}")
    return out[: n.value].copy()


def eigmap(img, block_size=3, use_harris=False, k=0.04):
    img = c_u8(img)
    h, w = img.shape
    out = np.zeros((h, w), np.float32)
    lib().vo_o_eigmap(ptr(img), w, h, int(block_size), int(bool(use_harris)), float(k), ptr(out))
    return out


def pyrdown(img):
    img = c_u8(img)
    h, w = img.shape
    out = np.zeros(((h + 1) // 2, (w + 1) // 2), np.uint8)
    lib().vo_o_pyrdown(ptr(img), w, h, ptr(out))
    return out


def scharr(img):
    img = c_u8(img)
    h, w = img.shape
    out = np.zeros((h, w, 2), np.int16)
    lib().vo_o_scharr(ptr(img), w, h, ptr(out))
    return out


def pyr_maxlevel(w, h, win=(15, 15), max_level=3):
    return lib().vo_o_pyr_maxlevel(w, h, win[0], win[1], max_level)


def lk(prev, nxt, pts, win=(15, 15), max_level=3, criteria=(3, 30, 0.01), min_eig=1e-4):
    prev = c_u8(prev)
    nxt = c_u8(nxt)
    pts = c_f32(pts).reshape(-1, 2)
    n = pts.shape[0]
    h, w = prev.shape
    out = np.zeros((n, 2), np.float32)
    st = np.zeros((n,), np.uint8)
    err = np.zeros((n,), np.float32)
    rc = lib().vo_o_lk(ptr(prev), ptr(nxt), w, h, ptr(pts), n, ptr(out), ptr(st), ptr(err),
                       int(win[0]), int(win[1]), int(max_level), int(criteria[0]), int(criteria[1]),
                       float(criteria[2]), float(min_eig))
    if rc < 0:
        raise RuntimeError(f"vo_o_lk failed rc={rc}")
    return out, st, err


def triangulate(P1, P2, x1, x2):
    """x1, x2: (2, n) arrays as passed to cv2.triangulatePoints; returns (4, n)."""
    P1 = c_f64(P1)
    P2 = c_f64(P2)
    x1 = np.asarray(x1)
    dt = np.float64 if x1.dtype == np.float64 else np.float32
    x1 = np.ascontiguousarray(np.asarray(x1, dt).reshape(2, -1).T)
    x2 = np.ascontiguousarray(np.asarray(x2, dt).reshape(2, -1).T)
    n = x1.shape[0]
    out = np.zeros((4, n), dt)
    if dt == np.float32:
        lib().vo_o_triangulate(ptr(P1), ptr(P2), ptr(x1), ptr(x2), n, ptr(out))
    else:
        lib().vo_o_triangulate_d(ptr(P1), ptr(P2), ptr(x1), ptr(x2), n, ptr(out))
    return out


def rodrigues(src):
    src = c_f64(src)
    if src.size == 3:
        R = np.zeros((3, 3), np.float64)
        lib().vo_o_rodrigues_v2m(ptr(src.reshape(3)), ptr(R))
        return R
    r = np.zeros((3, 1), np.float64)
    lib().vo_o_rodrigues_m2v(ptr(src.reshape(3, 3)), ptr(r))
    return r


def pnp_ransac_p3p(obj, img, K, iterations, reproj_err, confidence):
    obj = c_f32(obj).reshape(-1, 3)
    img = c_f32(img).reshape(-1, 2)
    K = c_f64(K)
    n = obj.shape[0]
    rvec = np.zeros((3, 1))
    tvec = np.zeros((3, 1))
    inl = np.zeros((max(n, 1),), np.int32)
    n_inl = C.c_int(0)
    succ = C.c_int(0)
    iters = C.c_int(0)
    rc = lib().vo_o_pnp_ransac_p3p(ptr(obj), ptr(img), n, ptr(K), int(iterations), float(reproj_err),
                                   float(confidence), ptr(rvec), ptr(tvec), ptr(inl), C.byref(n_inl),
                                   C.byref(succ), C.byref(iters))
    if rc < 0:
        raise RuntimeError(f"vo_o_pnp_ransac_p3p failed rc={rc}")
    return bool(succ.value), rvec, tvec, inl[: n_inl.value].copy(), iters.value


def p3p(K, obj4, img4):
    R = np.zeros((3, 3))
    t = np.zeros(3)
    ok = lib().vo_o_p3p(ptr(c_f64(K)), ptr(c_f64(obj4)), ptr(c_f64(img4)), ptr(R), ptr(t))
    return bool(ok), R, t


def epnp(K, obj, img):
    obj = c_f64(obj).reshape(-1, 3)
    img = c_f64(img).reshape(-1, 2)
    R = np.zeros((3, 3))
    t = np.zeros(3)
    ok = lib().vo_o_epnp(ptr(c_f64(K)), ptr(obj), ptr(img), obj.shape[0], ptr(R), ptr(t))
    return bool(ok), R, t


def find_essential(p0, p1, K, prob=0.999, threshold=1.0, max_iters=1000):
    p0 = c_f32(p0).reshape(-1, 2)
    p1 = c_f32(p1).reshape(-1, 2)
    n = p0.shape[0]
    E = np.zeros((3, 3))
    mask = np.zeros((max(n, 1),), np.uint8)
    nm = C.c_int(0)
    rc = lib().vo_o_find_essential(ptr(p0), ptr(p1), n, ptr(c_f64(K)), float(prob), float(threshold),
                                   int(max_iters), ptr(E), ptr(mask), C.byref(nm))
    return rc == 0, E, mask[:n].copy()


def five_point(q1, q2):
    E10 = np.zeros((10, 9))
    n = lib().vo_o_five_point(ptr(c_f64(q1)), ptr(c_f64(q2)), ptr(E10))
    return E10[:n].reshape(-1, 3, 3)


def recover_pose(E, p0, p1, K):
    p0 = c_f32(p0).reshape(-1, 2)
    p1 = c_f32(p1).reshape(-1, 2)
    n = p0.shape[0]
    R = np.zeros((3, 3))
    t = np.zeros((3, 1))
    mask = np.zeros((max(n, 1),), np.uint8)
    ng = C.c_int(0)
    lib().vo_o_recover_pose(ptr(c_f64(E)), ptr(p0), ptr(p1), n, ptr(c_f64(K)), ptr(R), ptr(t), ptr(mask),
                            C.byref(ng))
    return ng.value, R, t, mask[:n].copy()


def sift(img, cap=None, nfeatures=0):
    """SIFT_create(nfeatures).detectAndCompute(img, None): (kp [n,6], desc [n,128])."""
    img = c_u8(img)
    h, w = img.shape
    n = C.c_int(0)
    cap = 32768 if cap is None else int(cap)
    while True:
        kp = np.zeros((max(cap, 1), 6), np.float32)
        desc = np.zeros((max(cap, 1), 128), np.float32)
        lib().vo_o_sift_n(ptr(img), w, h, int(nfeatures), ptr(kp), ptr(desc), cap, C.byref(n))
        if n.value <= cap:
            return kp[:n.value].copy(), desc[:n.value].copy()
        cap = n.value


def retain_best(response, n_points):
    """KeyPointsFilter::retainBest on a response array: (perm [n] i32, kept)."""
    r = c_f32(response).reshape(-1)
    perm = np.zeros((max(len(r), 1),), np.int32)
    kept = lib().vo_o_retain_best(ptr(r), len(r), int(n_points), ptr(perm))
    if kept < 0:
        raise RuntimeError("vo_o_retain_best failed")
    return perm[:len(r)].copy(), int(kept)


def bf_knn2(q, t):
    q = c_f32(q)
    t = c_f32(t)
    nq, dim = q.shape
    nt = t.shape[0]
    idx = np.zeros((max(nq, 1), 2), np.int32)
    dist = np.zeros((max(nq, 1), 2), np.float32)
    lib().vo_o_bf_knn2(ptr(q), nq, ptr(t), nt, dim, ptr(idx), ptr(dist))
    return idx[:nq].copy(), dist[:nq].copy()
