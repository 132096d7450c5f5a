"""The reference's cv2 call surface, executed by libvo_hip.so on the GPU (boundary B1).

Same names, argument meanings, dtypes and output shapes as the OpenCV 4.6 calls made by
/root/reference/VisualOdometryPipeLine.py:

    goodFeaturesToTrack   :256        calcOpticalFlowPyrLK  :281,:287
    solvePnPRansac (P3P)  :343        Rodrigues             :354
    triangulatePoints     :188        SIFT_create / detectAndCompute :35,:226-227
    BFMatcher.knnMatch    :36,:229    findEssentialMat      :308
    recoverPose           :315

Each call copies numpy inputs to the device, runs the HIP kernels and copies results
back (the drop-in mode; the device-resident path is engine.Engine).  Installing this
module as ``sys.modules['cv2']`` lets the reference class itself run on the GPU.
There is no CPU fallback: every function raises if the HIP library is unavailable.
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np
import torch

from . import _lib as L
from .engine import Engine, make_opts

RANSAC = 8
LMEDS = 4
SOLVEPNP_ITERATIVE = 0
SOLVEPNP_EPNP = 1
SOLVEPNP_P3P = 2
TERM_CRITERIA_COUNT = 1
TERM_CRITERIA_MAX_ITER = 1
TERM_CRITERIA_EPS = 2
IMREAD_GRAYSCALE = 0
NORM_L2 = 4


class error(Exception):
    """Mirror of cv2.error."""


def _dev():
    if not torch.cuda.is_available():
        raise RuntimeError("cv2compat needs a ROCm GPU (no CPU fallback)")
    return torch.device("cuda")


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _p(t: torch.Tensor):
    return C.c_void_p(t.data_ptr())


_DEFAULT_OPTS = {
    "min_dist_landmarks": 1, "max_dist_landmarks": 150, "min_baseline_angle": 2, "min_baseline_frames": 2,
    "feature_ratio": 0.8, "feature_max_corners": 1400, "feature_quality_level": 0.1, "feature_min_dist": 10,
    "feature_block_size": 3, "feature_use_harris": False, "winSize": (21, 21), "maxLevel": 3,
    "criteria": (3, 30, 0.01), "PnP_conf": 0.99, "PnP_error": 8.0, "PnP_iterations": 100,
}

_ENGINES: dict = {}


def _engine(W, H, **over):
    key = (W, H, tuple(sorted((k, v if not isinstance(v, list) else tuple(v)) for k, v in over.items())))
    eng = _ENGINES.get(key)
    if eng is None:
        opts = dict(_DEFAULT_OPTS)
        opts.update(over)
        eng = Engine(np.eye(3), opts, W, H, batch=1, ncap=256, pcap=256, fcap=4)
        _ENGINES[key] = eng
    return eng


def _gray(img):
    a = np.asarray(img)
    if a.dtype != np.uint8 or a.ndim != 2:
        raise error("expected a uint8 grayscale image (CV_8UC1)")
    return np.ascontiguousarray(a)


# ---------------------------------------------------------------- GFTT (:256)
def goodFeaturesToTrack(image, maxCorners, qualityLevel, minDistance, mask=None, blockSize=3,
                        useHarrisDetector=False, k=0.04):
    if mask is not None:
        raise NotImplementedError("mask is not used by the reference (:256 passes None)")
    img = _gray(image)
    H, W = img.shape
    eng = _engine(W, H, feature_max_corners=int(maxCorners), feature_quality_level=float(qualityLevel),
                  feature_min_dist=float(minDistance), feature_block_size=int(blockSize),
                  feature_use_harris=bool(useHarrisDetector))
    eng.opts.harris_k = float(k)
    eng.t["status"].zero_()
    eng.build_pyramid(img, 0)
    L.check(eng.lib.vo_gftt(eng._pd, eng._po, eng._ps, 0, _stream()), "vo_gftt")
    st = int(eng.t["status"][0])
    if st != 0:
        raise error(L.STATUS_NAMES.get(st, str(st)))
    n = int(eng.t["nCorners"][0])
    if n == 0:
        return None
    return eng.t["corners"][0, :n].cpu().numpy().reshape(-1, 1, 2).copy()


# ---------------------------------------------------------------- LK (:281,:287)
def calcOpticalFlowPyrLK(prevImg, nextImg, prevPts, nextPts, winSize=(21, 21), maxLevel=3,
                         criteria=(TERM_CRITERIA_COUNT | TERM_CRITERIA_EPS, 30, 0.01), flags=0,
                         minEigThreshold=1e-4):
    if flags != 0 or nextPts is not None:
        raise NotImplementedError("OPTFLOW_USE_INITIAL_FLOW / flags are not used by the reference")
    p = np.asarray(prevPts)
    if p.dtype != np.float32:
        raise error("prevPts must be float32 (checkVector(2, CV_32F))")
    shape = p.shape
    pts = np.ascontiguousarray(p.reshape(-1, 2))
    n = pts.shape[0]
    a, b = _gray(prevImg), _gray(nextImg)
    if a.shape != b.shape:
        raise error("prevImg and nextImg must have the same size")
    H, W = a.shape
    eng = _engine(W, H, winSize=tuple(int(v) for v in winSize), maxLevel=int(maxLevel),
                  criteria=tuple(criteria))
    eng.opts.min_eig = float(minEigThreshold)
    eng.build_pyramid(a, 0)
    eng.build_pyramid(b, 1)
    dev = _dev()
    if n == 0:
        return np.zeros(shape, np.float32), np.zeros((0, 1), np.uint8), np.zeros((0, 1), np.float32)
    dp = torch.from_numpy(pts).to(dev).reshape(1, n, 2)
    cnt = torch.tensor([n], dtype=torch.int32, device=dev)
    out = torch.empty((1, n, 2), dtype=torch.float32, device=dev)
    st = torch.empty((1, n), dtype=torch.uint8, device=dev)
    err = torch.empty((1, n), dtype=torch.float32, device=dev)
    L.check(eng.lib.vo_lk_points(eng._pd, eng._po, eng._ps, 0, _p(dp), _p(cnt), n, _p(out), _p(st), _p(err),
                                 _stream()), "vo_lk_points")
    return (out.cpu().numpy().reshape(shape), st.cpu().numpy().reshape(-1, 1),
            err.cpu().numpy().reshape(-1, 1))


# ---------------------------------------------------------------- PnP (:343)
def solvePnPRansac(objectPoints, imagePoints, cameraMatrix, distCoeffs, rvec=None, tvec=None,
                   useExtrinsicGuess=False, iterationsCount=100, reprojectionError=8.0,
                   confidence=0.99, inliers=None, flags=SOLVEPNP_ITERATIVE):
    if flags != SOLVEPNP_P3P or useExtrinsicGuess:
        raise NotImplementedError("the reference uses flags=SOLVEPNP_P3P (:343)")
    if distCoeffs is not None and np.any(np.asarray(distCoeffs) != 0):
        raise NotImplementedError("non-zero distortion")
    obj = np.ascontiguousarray(np.asarray(objectPoints, np.float32).reshape(-1, 3))
    img = np.ascontiguousarray(np.asarray(imagePoints, np.float32).reshape(-1, 2))
    n = obj.shape[0]
    if n < 4 or img.shape[0] != n:
        raise error("solvePnPRansac: npoints >= 4 && npoints == ipoints required")
    opts = dict(_DEFAULT_OPTS, PnP_conf=float(confidence), PnP_error=float(reprojectionError),
                PnP_iterations=int(iterationsCount))
    o = make_opts(np.asarray(cameraMatrix, np.float64), opts)
    dev = _dev()
    d_obj = torch.from_numpy(obj).to(dev)
    d_img = torch.from_numpy(img).to(dev)
    cnt = torch.tensor([n], dtype=torch.int32, device=dev)
    rv = torch.zeros(3, dtype=torch.float64, device=dev)
    tv = torch.zeros(3, dtype=torch.float64, device=dev)
    ok = torch.zeros(1, dtype=torch.int32, device=dev)
    mask = torch.zeros(n, dtype=torch.uint8, device=dev)
    ninl = torch.zeros(1, dtype=torch.int32, device=dev)
    ws = 12 * n + 64
    work = torch.empty(ws, dtype=torch.float64, device=dev)
    L.check(L.lib().vo_pnp_ransac(C.byref(o), 1, _p(d_obj), _p(d_img), _p(cnt), n, _p(rv), _p(tv), _p(ok),
                                  _p(mask), _p(ninl), _p(work), ws, _stream()), "vo_pnp_ransac")
    success = bool(ok.item())
    if not success:
        return False, rv.cpu().numpy().reshape(3, 1), tv.cpu().numpy().reshape(3, 1), None
    inl = np.nonzero(mask.cpu().numpy())[0].astype(np.int32).reshape(-1, 1)
    return True, rv.cpu().numpy().reshape(3, 1), tv.cpu().numpy().reshape(3, 1), inl


# ---------------------------------------------------------------- DLT (:188)
def triangulatePoints(projMatr1, projMatr2, projPoints1, projPoints2):
    x1 = np.asarray(projPoints1)
    if x1.dtype != np.float32:
        raise NotImplementedError("float32 points (the reference's dtype, Q10)")
    x1 = np.ascontiguousarray(x1.reshape(2, -1).T)
    x2 = np.ascontiguousarray(np.asarray(projPoints2, np.float32).reshape(2, -1).T)
    n = x1.shape[0]
    dev = _dev()
    P1 = torch.from_numpy(np.ascontiguousarray(np.asarray(projMatr1, np.float64).reshape(1, 12))).to(dev).expand(n, 12).contiguous()
    P2 = torch.from_numpy(np.ascontiguousarray(np.asarray(projMatr2, np.float64).reshape(1, 12))).to(dev).expand(n, 12).contiguous()
    a = torch.from_numpy(x1).to(dev)
    b = torch.from_numpy(x2).to(dev)
    out = torch.empty((n, 4), dtype=torch.float32, device=dev)
    L.check(L.lib().vo_triangulate_points(n, _p(P1), _p(P2), _p(a), _p(b), _p(out), _stream()), "vo_triangulate_points")
    return out.cpu().numpy().T.copy()


# ---------------------------------------------------------------- Rodrigues (:354)
def Rodrigues(src, dst=None, jacobian=None):
    s = np.asarray(src, np.float64)
    dev = _dev()
    if s.size == 3:
        inp = torch.from_numpy(np.ascontiguousarray(s.reshape(3))).to(dev)
        out = torch.empty(9, dtype=torch.float64, device=dev)
        L.check(L.lib().vo_rodrigues(1, 1, _p(inp), _p(out), _stream()), "vo_rodrigues")
        return out.cpu().numpy().reshape(3, 3), np.zeros((3, 9))
    if s.size != 9:
        raise error("Rodrigues expects a 3-vector or a 3x3 matrix")
    inp = torch.from_numpy(np.ascontiguousarray(s.reshape(9))).to(dev)
    out = torch.empty(3, dtype=torch.float64, device=dev)
    L.check(L.lib().vo_rodrigues(1, 0, _p(inp), _p(out), _stream()), "vo_rodrigues")
    return out.cpu().numpy().reshape(3, 1), np.zeros((9, 3))


# ---------------------------------------------------------------- SIFT / BF (:35-36, :226-229)
class KeyPoint:
    __slots__ = ("pt", "size", "angle", "response", "octave", "class_id")

    def __init__(self, x=0.0, y=0.0, size=0.0, angle=-1.0, response=0.0, octave=0, class_id=-1):
        self.pt = (float(x), float(y))
        self.size = float(size)
        self.angle = float(angle)
        self.response = float(response)
        self.octave = int(octave)
        self.class_id = int(class_id)


class DMatch:
    __slots__ = ("queryIdx", "trainIdx", "imgIdx", "distance")

    def __init__(self, queryIdx=-1, trainIdx=-1, imgIdx=0, distance=float(np.finfo(np.float32).max)):
        self.queryIdx = int(queryIdx)
        self.trainIdx = int(trainIdx)
        self.imgIdx = int(imgIdx)
        self.distance = float(distance)


_SIFTS: dict = {}


class _SIFT:
    def __init__(self, nfeatures: int = 0):
        self.nfeatures = int(nfeatures)

    def detectAndCompute(self, image, mask):
        from .features import Sift
        if mask is not None:
            raise NotImplementedError("mask is not used by the reference (:226 passes None)")
        img = _gray(image)
        H, W = img.shape
        s = _SIFTS.get((W, H, self.nfeatures))
        if s is None:
            s = _SIFTS[(W, H, self.nfeatures)] = Sift(W, H, _dev(), nfeatures=self.nfeatures)
        s.run(torch.from_numpy(img).to(_dev()))
        kp, desc = s.result()
        kps = tuple(KeyPoint(k[0], k[1], k[2], k[3], k[4], int(k[5])) for k in kp)
        return kps, (desc.copy() if len(kps) else None)


def SIFT_create(nfeatures=0, *args, **kwargs):
    """SIFT_create() (:35) or SIFT_create(nfeatures) (KeyPointsFilter::retainBest cap, BASELINE C5);
    the other SIFT parameters keep OpenCV's defaults."""
    if args or kwargs or int(nfeatures) < 0:
        raise NotImplementedError("only nfeatures may be set (the reference uses the default SIFT, :35)")
    return _SIFT(nfeatures)


class _BFMatcher:
    def knnMatch(self, queryDescriptors, trainDescriptors, k=2):
        from .features import bf_knn2
        if k != 2:
            raise NotImplementedError("the reference uses k=2 (:229)")
        q = np.ascontiguousarray(np.asarray(queryDescriptors, np.float32))
        t = np.ascontiguousarray(np.asarray(trainDescriptors, np.float32))
        if q.ndim != 2 or q.shape[1] != 128 or t.shape[1] != 128:
            raise NotImplementedError("128-D float descriptors (SIFT)")
        if not (np.array_equal(q, np.round(q)) and np.array_equal(t, np.round(t))):
            raise NotImplementedError("the MFMA matcher is exact for integer-valued (SIFT) descriptors")
        # the int8 kernel stores v - 128: exact for 0..255 (SIFT's saturate_cast<uchar> range),
        # anything outside would wrap into a wrong distance
        if (q.size and (q.min() < 0 or q.max() > 255)) or (t.size and (t.min() < 0 or t.max() > 255)):
            raise NotImplementedError("the MFMA matcher takes descriptor values 0..255 (SIFT)")
        dev = _dev()
        nq, nt = q.shape[0], t.shape[0]
        if nq == 0:
            return ()
        dq = torch.from_numpy(q).to(dev)
        dt = torch.from_numpy(t if nt else np.zeros((1, 128), np.float32)).to(dev)
        cq = torch.tensor([nq], dtype=torch.int32, device=dev)
        ct = torch.tensor([nt], dtype=torch.int32, device=dev)
        idx2, dist2 = bf_knn2(dq, cq, dt, ct, nq)
        idx2 = idx2.cpu().numpy()
        dist2 = dist2.cpu().numpy()
        out = []
        for i in range(nq):
            out.append(tuple(DMatch(i, int(idx2[i, j]), 0, float(dist2[i, j])) for j in range(2) if idx2[i, j] >= 0))
        return tuple(out)


def BFMatcher(normType=NORM_L2, crossCheck=False):
    if normType != NORM_L2 or crossCheck:
        raise NotImplementedError
    return _BFMatcher()


# ---------------------------------------------------------------- E / pose (:308, :315)
def findEssentialMat(points1, points2, cameraMatrix, method=RANSAC, prob=0.999, threshold=1.0, maxIters=1000,
                     mask=None):
    if method != RANSAC:
        raise NotImplementedError("the reference uses RANSAC (:308)")
    p0 = np.ascontiguousarray(np.asarray(points1, np.float32).reshape(-1, 2))
    p1 = np.ascontiguousarray(np.asarray(points2, np.float32).reshape(-1, 2))
    n = p0.shape[0]
    if p1.shape[0] != n:
        raise error("points1 and points2 must have the same size")
    o = make_opts(np.asarray(cameraMatrix, np.float64), _DEFAULT_OPTS)
    dev = _dev()
    a = torch.from_numpy(p0 if n else np.zeros((1, 2), np.float32)).to(dev)
    b = torch.from_numpy(p1 if n else np.zeros((1, 2), np.float32)).to(dev)
    cap = max(n, 1)
    cnt = torch.tensor([n], dtype=torch.int32, device=dev)
    E = torch.zeros(9, dtype=torch.float64, device=dev)
    m = torch.zeros(cap, dtype=torch.uint8, device=dev)
    ok = torch.zeros(1, dtype=torch.int32, device=dev)
    ws = 4 * cap + 90 * 64 + 64
    work = torch.empty(ws, dtype=torch.float64, device=dev)
    L.check(L.lib().vo_find_essential(C.byref(o), 1, _p(a), _p(b), _p(cnt), cap, float(prob), float(threshold),
                                      int(maxIters), _p(E), _p(m), _p(ok), _p(work), ws, _stream()),
            "vo_find_essential")
    mk = m.cpu().numpy()[:n].reshape(-1, 1)
    if not int(ok.item()):
        return None, mk
    return E.cpu().numpy().reshape(3, 3), mk


def recoverPose(E, points1, points2, cameraMatrix, *args, **kwargs):
    if args or kwargs:
        raise NotImplementedError("the reference passes (E, p0, p1, K) only (:315)")
    p0 = np.ascontiguousarray(np.asarray(points1, np.float32).reshape(-1, 2))
    p1 = np.ascontiguousarray(np.asarray(points2, np.float32).reshape(-1, 2))
    n = p0.shape[0]
    o = make_opts(np.asarray(cameraMatrix, np.float64), _DEFAULT_OPTS)
    dev = _dev()
    cap = max(n, 1)
    a = torch.from_numpy(p0 if n else np.zeros((1, 2), np.float32)).to(dev)
    b = torch.from_numpy(p1 if n else np.zeros((1, 2), np.float32)).to(dev)
    cnt = torch.tensor([n], dtype=torch.int32, device=dev)
    dE = torch.from_numpy(np.ascontiguousarray(np.asarray(E, np.float64).reshape(9))).to(dev)
    R = torch.zeros(9, dtype=torch.float64, device=dev)
    t = torch.zeros(3, dtype=torch.float64, device=dev)
    m = torch.zeros(cap, dtype=torch.uint8, device=dev)
    ng = torch.zeros(1, dtype=torch.int32, device=dev)
    L.check(L.lib().vo_recover_pose(C.byref(o), 1, _p(dE), _p(a), _p(b), _p(cnt), cap, _p(R), _p(t), _p(m), _p(ng),
                                    _stream()), "vo_recover_pose")
    return (int(ng.item()), R.cpu().numpy().reshape(3, 3), t.cpu().numpy().reshape(3, 1),
            (m.cpu().numpy()[:n].reshape(-1, 1) * 255).astype(np.uint8))
