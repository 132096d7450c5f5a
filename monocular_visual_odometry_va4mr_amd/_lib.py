"""ctypes binding of libvo_hip.so (include/vo_hip.h).

The library is built in-tree (``__graft_entry__.build()`` or ``make -C csrc``) into
``monocular_visual_odometry_va4mr_amd/_build/libvo_hip.so``.  There is no CPU fallback:
if the library or a GPU is missing, :func:`lib` raises.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VO_HIP_LIB") or os.path.join(_HERE, "_build", "libvo_hip.so")
CSRC = os.path.join(_HERE, "csrc")

VO_MAX_LEVELS = 8
VO_BORDER = 16

ST_OK = 0
ST_NOT_ENOUGH_KP = 1
ST_PNP_FAILED = 2
ST_GFTT_NONE = 3
ST_GFTT_ONE = 4
ST_CAPACITY = 5
ST_ESSENTIAL_FAILED = 6
ST_NO_MATCHES = 7

STATUS_NAMES = {
    ST_OK: "ok",
    ST_NOT_ENOUGH_KP: "Not enough keypoints for PnP",
    ST_PNP_FAILED: "PnP failed",
    ST_GFTT_NONE: "goodFeaturesToTrack returned no corners",
    ST_GFTT_ONE: "goodFeaturesToTrack returned a single corner",
    ST_CAPACITY: "engine capacity exceeded",
    ST_ESSENTIAL_FAILED: "findEssentialMat found no model",
    ST_NO_MATCHES: "no bootstrap matches",
}

i32, i64, f64, vp = C.c_int32, C.c_int64, C.c_double, C.c_void_p


class VoDims(C.Structure):
    _fields_ = [
        ("B", i32), ("W", i32), ("H", i32), ("nlev", i32),
        ("lvl_w", i32 * VO_MAX_LEVELS), ("lvl_h", i32 * VO_MAX_LEVELS), ("lvl_pitch", i32 * VO_MAX_LEVELS),
        ("lvl_off", i64 * VO_MAX_LEVELS),
        ("pyr_stride", i64), ("der_stride", i64),
        ("ncap", i32), ("pcap", i32), ("fcap", i32), ("ccap", i32), ("mcap", i32),
        ("work_stride", i64), ("iwork_stride", i64),
    ]


class VoOpts(C.Structure):
    _fields_ = [
        ("K", f64 * 9), ("K_inv", f64 * 9),
        ("min_dist_landmarks", f64), ("max_dist_landmarks", f64),
        ("min_baseline_angle", f64), ("cos_baseline", f64),
        ("min_baseline_frames", i32),
        ("feature_ratio", f64),
        ("feature_max_corners", i32),
        ("feature_quality_level", f64), ("feature_min_dist", f64),
        ("feature_block_size", i32), ("feature_use_harris", i32),
        ("harris_k", f64),
        ("win_w", i32), ("win_h", i32), ("max_level", i32), ("crit_type", i32), ("crit_count", i32),
        ("crit_eps", f64), ("min_eig", f64),
        ("pnp_conf", f64), ("pnp_error", f64),
        ("pnp_iters", i32),
    ]


_STATE_FIELDS = [
    "pyr0", "pyr1", "der0", "der1", "lm_X", "lm_kp", "nL", "c_kp", "c_first", "c_tau", "nC",
    "pose_R", "pose_t", "nF", "num_pts", "outl_kp", "inl_kp", "nOutl", "nInl", "status",
    "trk_pts", "trk_st", "trk_err", "eig", "eig_max", "gf_keys", "gf_n", "corners", "nCorners",
    "pnp_rt", "pnp_ok", "pnp_ninl", "pnp_mask", "work", "iwork", "gf_sort",
]

VO_GF_SORT_EXTRA = 4096


class VoState(C.Structure):
    _fields_ = [(n, vp) for n in _STATE_FIELDS]


VO_SIFT_MAX_OCT = 16


class VoSiftBuf(C.Structure):
    _fields_ = [
        ("W", i32), ("H", i32), ("n_oct", i32),
        ("oct_w", i32 * VO_SIFT_MAX_OCT), ("oct_h", i32 * VO_SIFT_MAX_OCT),
        ("gauss_off", i64 * (VO_SIFT_MAX_OCT * 6)), ("dog_off", i64 * (VO_SIFT_MAX_OCT * 5)),
        ("gauss_floats", i64), ("dog_floats", i64), ("tmp_floats", i64),
        ("gauss", vp), ("dog", vp), ("tmp", vp), ("consts", vp), ("counters", vp), ("cand", vp),
        ("kp", vp), ("kp_out", vp), ("desc", vp), ("hist", vp),
        ("cand_cap", i32), ("kp_cap", i32), ("nfeatures", i32),
    ]


_lib = None


def build(verbose: bool = False) -> str:
    """Compile libvo_hip.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    jobs = str(min(16, os.cpu_count() or 4))
    out = subprocess.run(["make", "-s", "-j", jobs, "-C", CSRC], capture_output=not verbose, text=True)
    if out.returncode != 0:
        raise RuntimeError("building libvo_hip.so failed:\n" + (out.stderr or "")[-4000:])
    return LIB_PATH


def lib():
    """Load libvo_hip.so (never falls back to a CPU path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: run __graft_entry__.build() (no CPU fallback exists)")
        _lib = C.CDLL(LIB_PATH)
        _declare(_lib)
    return _lib


def _declare(L):
    P = vp
    D = C.POINTER(VoDims)
    O = C.POINTER(VoOpts)
    S = C.POINTER(VoState)
    sig = {
        "vo_version": ([], C.c_char_p),
        "vo_device_arch": ([C.c_char_p, C.c_int], C.c_int),
        "vo_device_cus": ([], C.c_int),
        "vo_set_launch_cus": ([C.c_int], C.c_int),
        "vo_set_gftt_select": ([C.c_int], C.c_int),
        "vo_stream_create_cumask": ([C.c_int, C.c_int, C.POINTER(C.c_void_p)], C.c_int),
        "vo_stream_destroy": ([P], C.c_int),
        "vo_pyr_build": ([D, S, C.c_int, P, i64, P], C.c_int),
        "vo_pyr_deriv": ([D, S, C.c_int, P], C.c_int),
        "vo_track": ([D, O, S, C.c_int, P], C.c_int),
        "vo_track_lk": ([D, O, S, C.c_int, P], C.c_int),
        "vo_pnp": ([D, O, S, P], C.c_int),
        "vo_triangulate": ([D, O, S, C.c_int, P], C.c_int),
        "vo_pnp_triangulate": ([D, O, S, P], C.c_int),
        "vo_filter_pnp_triangulate": ([D, O, S, P], C.c_int),
        "vo_gftt": ([D, O, S, C.c_int, P], C.c_int),
        "vo_gftt_eigmap": ([D, O, S, C.c_int, P], C.c_int),
        "vo_add_corners_finish": ([D, O, S, P], C.c_int),
        "vo_status_word": ([S, P, P], C.c_int),
        "vo_lk_points": ([D, O, S, C.c_int, P, P, i32, P, P, P, P], C.c_int),
        "vo_pnp_ransac": ([O, C.c_int, P, P, P, i32, P, P, P, P, P, P, i64, P], C.c_int),
        "vo_triangulate_points": ([C.c_int, P, P, P, P, P, P], C.c_int),
        "vo_rodrigues": ([C.c_int, C.c_int, P, P, P], C.c_int),
    }
    SB = C.POINTER(VoSiftBuf)
    optional = {
        "vo_sift_plan": ([SB, C.c_int, C.c_int], C.c_int),
        "vo_sift": ([SB, P, C.c_int, C.c_int, P], C.c_int),
        "vo_sift_batch": ([SB, C.c_int, P, C.c_int64, C.c_int, C.c_int, P], C.c_int),
        "vo_sift_retain_best_rows": ([P, i32, i32, P, P, P, P], C.c_int),
        "vo_ratio_matches": ([C.c_int, P, P, i32, P, P, P, i32, f64, P, P, P, i32, P], C.c_int),
        "vo_find_essential": ([O, C.c_int, P, P, P, i32, f64, f64, i32, P, P, P, P, i32, P], C.c_int),
        "vo_recover_pose": ([O, C.c_int, P, P, P, P, i32, P, P, P, P, P], C.c_int),
        "vo_bootstrap": ([D, O, S, P, P, P, i32, P], C.c_int),
        "vo_bf_knn2_batch_scratch": ([C.c_int, i32, i32], i64),
        "vo_bf_knn2_batch": ([C.c_int, P, P, i32, P, P, i32, i32, P, P, P, i64, P], C.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    for name, (args, res) in optional.items():
        if hasattr(L, name):
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res


def exported_symbols():
    """Symbols declared in include/vo_hip.h (used by the CPU-side ABI test)."""
    import re
    hdr = os.path.join(os.path.dirname(_HERE), "include", "vo_hip.h")
    txt = open(hdr).read()
    return sorted(set(re.findall(r"^\s*(?:const char\*|int|int64_t)\s+(vo_\w+)\s*\(", txt, re.M)))


def check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"{what} failed with status {rc}")
