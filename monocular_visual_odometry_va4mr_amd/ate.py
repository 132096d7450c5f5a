"""Absolute trajectory error: Umeyama Sim(3) alignment + RMSE.

The reference defines no accuracy metric (README.md has a qualitative plot only); the
build's parity bar is: camera positions p_k = transforms[k][1] of the MI355X path,
Sim(3)-aligned to the reference CPU path's positions, RMSE <= 1% of the reference path
length.
"""
from __future__ import annotations

import numpy as np


def umeyama(src: np.ndarray, dst: np.ndarray, with_scale: bool = True):
    """Least-squares s, R, t with dst ~ s R src + t (Umeyama 1991).  src, dst: (n, 3)."""
    src = np.asarray(src, np.float64)
    dst = np.asarray(dst, np.float64)
    mu_s, mu_d = src.mean(0), dst.mean(0)
    xs, xd = src - mu_s, dst - mu_d
    n = src.shape[0]
    cov = xd.T @ xs / n
    U, D, Vt = np.linalg.svd(cov)
    S = np.eye(3)
    if np.linalg.det(U) * np.linalg.det(Vt) < 0:
        S[2, 2] = -1
    R = U @ S @ Vt
    var_s = (xs ** 2).sum() / n
    s = (D * np.diag(S)).sum() / var_s if (with_scale and var_s > 0) else 1.0
    t = mu_d - s * R @ mu_s
    return s, R, t


def path_length(p: np.ndarray) -> float:
    p = np.asarray(p, np.float64)
    return float(np.linalg.norm(np.diff(p, axis=0), axis=1).sum()) if len(p) > 1 else 0.0


def ate(est: np.ndarray, ref: np.ndarray, with_scale: bool = True):
    """Returns (rmse, rmse / path_length(ref)) after aligning est onto ref."""
    est = np.asarray(est, np.float64).reshape(-1, 3)
    ref = np.asarray(ref, np.float64).reshape(-1, 3)
    n = min(len(est), len(ref))
    est, ref = est[:n], ref[:n]
    if n < 3:
        d = est - ref
        rmse = float(np.sqrt((d ** 2).sum(1).mean())) if n else 0.0
        return rmse, rmse / max(path_length(ref), 1e-12)
    s, R, t = umeyama(est, ref, with_scale)
    al = (s * (R @ est.T)).T + t
    rmse = float(np.sqrt(((al - ref) ** 2).sum(1).mean()))
    return rmse, rmse / max(path_length(ref), 1e-12)
