"""``cv2``-compatible CPU shim over the C oracle (test infrastructure only).

Implements exactly the cv2 surface the reference uses:
SIFT_create/detectAndCompute (VisualOdometryPipeLine.py:35,226-227), BFMatcher/knnMatch
(:36,229), goodFeaturesToTrack (:256), calcOpticalFlowPyrLK (:281,287), findEssentialMat
(:308), recoverPose (:315), solvePnPRansac with SOLVEPNP_P3P (:343), triangulatePoints
(:188), Rodrigues (:354) and the constants used at :308,:343 and main.py:38.

Injected as ``sys.modules['cv2']`` it lets the *reference's own*
``VisualOdometryPipeLine`` class run in this container, which is how the golden
fixtures under tests/golden are produced (tests/golden/make_golden.py).
"""
from __future__ import annotations

import numpy as np

from . import _olib as O

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

__version__ = "4.6.0-oracle"


class error(Exception):
    """Mirror of cv2.error (OpenCV assertion failures)."""


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


class _SIFT:
    def __init__(self, nfeatures=0):
        self.nfeatures = int(nfeatures)

    def detectAndCompute(self, image, mask):
        if mask is not None:
            raise NotImplementedError("mask not supported (the reference passes None)")
        img = np.asarray(image)
        if img.ndim != 2 or img.dtype != np.uint8:
            raise error("SIFT oracle expects a uint8 grayscale image")
        kp, desc = O.sift(img, nfeatures=self.nfeatures)
        kps = tuple(KeyPoint(k[0], k[1], k[2], k[3], k[4], int(k[5])) for k in kp)
        return kps, (desc if len(kps) else None)


def SIFT_create(nfeatures=0, *args, **kwargs):
    if args or kwargs or int(nfeatures) < 0:
        raise NotImplementedError("only nfeatures may be set (the reference uses the default SIFT, :35)")
    return _SIFT(nfeatures)


class _BFMatcher:
    def knnMatch(self, queryDescriptors, trainDescriptors, k=2):
        if k != 2:
            raise NotImplementedError("reference uses k=2 (:229)")
        q = np.asarray(queryDescriptors, np.float32)
        t = np.asarray(trainDescriptors, np.float32)
        idx, dist = O.bf_knn2(q, t)
        out = []
        for i in range(q.shape[0]):
            row = []
            for j in range(2):
                if idx[i, j] >= 0:
                    row.append(DMatch(i, int(idx[i, j]), 0, float(dist[i, j])))
            out.append(tuple(row))
        return tuple(out)


def BFMatcher(normType=NORM_L2, crossCheck=False):
    if normType != NORM_L2 or crossCheck:
        raise NotImplementedError
    return _BFMatcher()


def goodFeaturesToTrack(image, maxCorners, qualityLevel, minDistance, mask=None, blockSize=3,
                        useHarrisDetector=False, k=0.04):
    if mask is not None:
        raise NotImplementedError
    img = np.asarray(image)
    if img.dtype != np.uint8 or img.ndim != 2:
        raise error("goodFeaturesToTrack oracle expects uint8 grayscale")
    pts = O.gftt(img, maxCorners, qualityLevel, minDistance, blockSize, useHarrisDetector, k)
    if pts.shape[0] == 0:
        return None
    return pts.reshape(-1, 1, 2)


def calcOpticalFlowPyrLK(prevImg, nextImg, prevPts, nextPts, winSize=(21, 21), maxLevel=3,
                         criteria=(TERM_CRITERIA_COUNT | TERM_CRITERIA_EPS, 30, 0.01), flags=0,
                         minEigThreshold=1e-4):
    if flags != 0:
        raise NotImplementedError
    p = np.asarray(prevPts)
    if p.dtype != np.float32:
        raise error("prevPts must be float32 (checkVector(2, CV_32F))")
    shape = p.shape
    out, st, err = O.lk(prevImg, nextImg, p.reshape(-1, 2), tuple(winSize), int(maxLevel),
                        tuple(criteria), float(minEigThreshold))
    return out.reshape(shape), st.reshape(-1, 1), err.reshape(-1, 1)


def findEssentialMat(points1, points2, cameraMatrix, method=RANSAC, prob=0.999, threshold=1.0,
                     maxIters=1000, mask=None):
    if method != RANSAC:
        raise NotImplementedError
    p0 = np.asarray(points1, np.float32).reshape(-1, 2)
    p1 = np.asarray(points2, np.float32).reshape(-1, 2)
    ok, E, m = O.find_essential(p0, p1, cameraMatrix, prob, threshold, maxIters)
    if not ok:
        return None, m.reshape(-1, 1)
    return E, m.reshape(-1, 1)


def recoverPose(E, points1, points2, cameraMatrix, *args, **kwargs):
    if args or kwargs:
        raise NotImplementedError
    ng, R, t, mask = O.recover_pose(E, points1, points2, cameraMatrix)
    return ng, R, t, (mask.reshape(-1, 1) * 255).astype(np.uint8)


def solvePnPRansac(objectPoints, imagePoints, cameraMatrix, distCoeffs, rvec=None, tvec=None,
                   useExtrinsicGuess=False, iterationsCount=100, reprojectionError=8.0,
                   confidence=0.99, inliers=None, flags=SOLVEPNP_ITERATIVE):
    if flags != SOLVEPNP_P3P or useExtrinsicGuess:
        raise NotImplementedError("oracle restates SOLVEPNP_P3P only (reference :343)")
    if distCoeffs is not None and np.any(np.asarray(distCoeffs) != 0):
        raise NotImplementedError("non-zero distortion")
    obj = np.asarray(objectPoints)
    img = np.asarray(imagePoints)
    n = obj.reshape(-1, 3).shape[0] if obj.size else 0
    if n < 4 or img.reshape(-1, 2).shape[0] != n:
        raise error("solvePnPRansac: npoints >= 4 && npoints == ipoints required")
    ok, rv, tv, inl, _ = O.pnp_ransac_p3p(obj, img, cameraMatrix, iterationsCount, reprojectionError,
                                         confidence)
    return ok, rv, tv, (inl.reshape(-1, 1) if ok else None)


def triangulatePoints(projMatr1, projMatr2, projPoints1, projPoints2):
    return O.triangulate(projMatr1, projMatr2, projPoints1, projPoints2)


def Rodrigues(src, dst=None, jacobian=None):
    src = np.asarray(src, np.float64)
    out = O.rodrigues(src)
    jac = np.zeros((3, 9) if src.size == 3 else (9, 3))
    return out, jac
