"""Which floating-point evaluation does this host's numpy/BLAS use for the small matrix
products of the reference's pose and triangulation code (VisualOdometryPipeLine.py:74-75,
:141-143, :157-168, :170-171)?  The kernels reproduce the models below (vo_pose.hip); run
this on any host whose numpy produced fixtures or oracle results (OpenBLAS picks kernels
by CPU).  Prints, per product kind, how many of n random cases each candidate model
reproduces bit for bit; exit code 1 if a model the kernels rely on does not hold."""
import itertools
import sys
from fractions import Fraction

import numpy as np


def fma(a, b, c):
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def dot_models():
    """3-term dot product evaluation orders: fma chains over every permutation, plain sums."""
    m = {}
    for p in itertools.permutations(range(3)):
        m["chain" + "".join(map(str, p))] = (lambda a, b, p=p: fma(a[p[2]], b[p[2]], fma(a[p[1]], b[p[1]], a[p[0]] * b[p[0]])))
    m["plain012"] = lambda a, b: (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]
    return m


def rot(rng):
    return np.ascontiguousarray(np.linalg.qr(rng.normal(size=(3, 3)))[0])


def main(n=600):
    rng = np.random.default_rng(0)
    models = dot_models()
    K = np.array([[718.856, 0, 607.1928], [0, 718.856, 185.2157], [0, 0, 1.0]])
    cases = {
        # name: (A builder, x builder, product) -- A's memory order is what numpy hands BLAS
        "gemv C-order A (-R_WC @ t, step poses)": lambda: (-(rot(rng).T.T), rng.normal(size=(3, 1)) * 10),
        "gemv F-order A (-R.T @ t, bootstrap/Rodrigues)": lambda: (-rot(rng).T, rng.normal(size=(3, 1)) * 10),
        "gemm K @ [R|t] (C x C, 3x4)": lambda: (K, np.hstack((rot(rng), rng.normal(size=(3, 1)) * 10))),
        "gemm R_cur.T @ R_past (C x F)": lambda: (np.asfortranarray(rot(rng)).T, np.asfortranarray(rot(rng))),
        "gemm R_cur.T @ R_past (C x C)": lambda: (np.asfortranarray(rot(rng)).T, rot(rng)),
        "gemm R_cur.T @ R_past (F x C)": lambda: (rot(rng).T, rot(rng)),
        "gemm rel @ K_inv (F x C)": lambda: (rot(rng).T, np.linalg.inv(K)),
    }
    score = {}
    for name, mk in cases.items():
        ok = {k: 0 for k in models}
        for _ in range(n):
            A, X = mk()
            ref = A @ X
            if not (A.ndim == 2 and X.shape[0] == 3):
                raise AssertionError(name)
            for k, f in models.items():
                v = np.array([[f(A[i], X[:, j]) for j in range(X.shape[1])] for i in range(3)])
                ok[k] += np.array_equal(v, ref)
        best = sorted(ok.items(), key=lambda kv: -kv[1])[:3]
        score[name] = dict(best)
        print(f"{name}: " + ", ".join(f"{k} {v}/{n}" for k, v in best))
    need = {"gemv C-order A (-R_WC @ t, step poses)": "chain102",
            "gemv F-order A (-R.T @ t, bootstrap/Rodrigues)": "chain012",
            "gemm K @ [R|t] (C x C, 3x4)": "chain012",
            "gemm R_cur.T @ R_past (C x F)": "chain012",
            "gemm R_cur.T @ R_past (C x C)": "chain012",
            "gemm R_cur.T @ R_past (F x C)": "chain012",
            "gemm rel @ K_inv (F x C)": "chain012"}
    bad = [k for k, m in need.items() if score[k].get(m, 0) != n]
    print("kernel models hold" if not bad else f"MODEL MISMATCH: {bad}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
