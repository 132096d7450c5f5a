"""Which floating-point evaluation does this host's numpy/BLAS use for the reference's
pose inversion ``tnew = -R.T @ t`` (VisualOdometryPipeLine.py:74-75)?

k_pnp_apply reproduces a column-major gemv accumulated with fused multiply-adds in
column order j = 0, 1, 2.  This probe checks that model against numpy on random rotations
(run it on the GPU box host too: OpenBLAS picks its kernels by CPU).  Exit code 1 if the
model does not hold."""
import sys
from fractions import Fraction

import numpy as np


def fma(a, b, c):
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def main(n=4000):
    rng = np.random.default_rng(0)
    ok = 0
    for _ in range(n):
        R = np.ascontiguousarray(np.linalg.qr(rng.normal(size=(3, 3)))[0])   # C-order, as Rodrigues returns
        t = rng.normal(size=(3, 1)) * rng.uniform(0.1, 100)
        Rn = R.T
        ref = (-Rn @ t)[:, 0]
        A = -Rn
        model = np.array([fma(A[i, 2], t[2, 0], fma(A[i, 1], t[1, 0], A[i, 0] * t[0, 0])) for i in range(3)])
        ok += np.array_equal(model, ref)
    print(f"blas_order_probe: column fma-chain model matches numpy on {ok}/{n} pose inversions")
    return 0 if ok == n else 1


if __name__ == "__main__":
    sys.exit(main())
