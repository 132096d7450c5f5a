"""The f32 fast paths k_lk_w uses for two of OpenCV's decisions (round 6) never decide differently
from the exact computation (csrc/vo_image.hip, k_lk_w; lkpyramid.cpp semantics):

* the minEig gate  (A22 + A11 - sqrtf(t)) / (2 WW WH) < min_eig  (correctly rounded f32 sqrt and
  division) is first decided from the raw v_sqrt_f32 (modelled here as the correctly rounded sqrt
  moved by up to 2 ulp either way) and a multiply by the reciprocal, with the margin
  mg = 2^-20 ((sa + sum) / 450 + |ma|) + 2^-100;
* the convergence test  fma((double)ddx, ddx, (double)ddy^2) <= eps^2  is first decided from
  fmaf(ddx, ddx, ddy * ddy) against eps2 (1 -+ 2^-20) (fill_lk's eps2_lo / eps2_hi).

The kernel falls back to the exact form whenever the fast form does not decide; here every case
the fast form does decide is checked against the exact decision, including inputs placed right
at the thresholds.  CPU only (numpy float32 / float64 arithmetic, no GPU).
"""
import numpy as np

F = np.float32
WW = WH = 15
N = 2 * WW * WH


def _fmaf(a, b, c):
    """float32 fma: the product exact in extended precision, one rounding to float32 (up to
    extended-precision double rounding, immaterial for these margins and steps)."""
    L = np.longdouble
    return np.float32(L(a) * L(b) + L(c))


def _ulp_shift(x, k):
    """x moved by k float32 ulps (k may be negative)."""
    x = np.asarray(x, np.float32)
    step = np.float32(np.inf) if k > 0 else np.float32(-np.inf)
    for _ in range(abs(k)):
        x = np.nextafter(x, step)
    return x


def _min_eig_exact(A11, A12, A22):
    t = (A11 - A22) * (A11 - A22) + F(4) * A12 * A12
    return (A22 + A11 - np.sqrt(t)) / F(N)


def _min_eig_fast(A11, A12, A22, thr, k):
    """The kernel's fast decision (1 reject / 0 accept / -1 left to the exact path), with the raw sqrt
    modelled as the correctly rounded one moved by k ulps."""
    t = (A11 - A22) * (A11 - A22) + F(4) * A12 * A12
    s2 = A22 + A11
    sa = _ulp_shift(np.sqrt(t), k)
    inv_n = F(1) / F(N)
    ma = (s2 - sa) * inv_n
    mg = _fmaf(F(2.0 ** -20), (sa + s2) * inv_n + np.abs(ma), F(2.0 ** -100))
    reject = ma + mg < thr
    accept = ma - mg >= thr
    return np.where(reject, 1, np.where(accept, 0, -1))


def test_min_eig_fast_gate_agrees_with_exact():
    rng = np.random.default_rng(7)
    n = 200_000
    # integer tensor sums x 2^-20 as the kernel forms them (a11, a22 >= 0, a11 a22 >= a12^2)
    a11 = rng.integers(0, 1 << 30, n).astype(np.float64)
    a22 = rng.integers(0, 1 << 30, n).astype(np.float64)
    r = rng.uniform(-1, 1, n)
    a12 = np.floor(r * np.sqrt(a11 * a22))
    A11, A12, A22 = (np.float32(v * 2.0 ** -20) for v in (a11, a12, a22))
    exact = _min_eig_exact(A11, A12, A22)
    for thr in (F(1e-4), F(1e-3), F(0.0)):
        ex = exact < thr
        for k in (-2, -1, 0, 1, 2):
            fast = _min_eig_fast(A11, A12, A22, thr, k)
            decided = fast >= 0
            assert np.array_equal(fast[decided] == 1, ex[decided]), (thr, k)
            assert np.mean(decided) > 0.99            # the exact path runs rarely
    # thresholds placed exactly at (and one ulp around) the exact value: the fast form must either
    # agree or leave the case to the exact path
    idx = rng.choice(n, 2000, replace=False)
    for d in (-1, 0, 1):
        thr = _ulp_shift(exact[idx], d)
        ex = exact[idx] < thr
        for k in (-2, 0, 2):
            fast = _min_eig_fast(A11[idx], A12[idx], A22[idx], thr, k)
            decided = fast >= 0
            assert np.array_equal(fast[decided] == 1, ex[decided])


def _eps_bounds(eps2):
    lo = np.nextafter(np.float32(eps2 * (1 - 2.0 ** -20)), np.float32(0))
    hi = np.nextafter(np.float32(eps2 * (1 + 2.0 ** -20)), np.float32(np.inf))
    return lo, hi


def test_convergence_fast_test_agrees_with_double():
    rng = np.random.default_rng(11)
    for eps in (0.01, 0.03, 1e-3, 0.5):
        eps2 = eps * eps
        lo, hi = _eps_bounds(eps2)
        n = 200_000
        # steps spread log-normally around the threshold radius
        ang = rng.uniform(0, 2 * np.pi, n)
        rad = eps * np.exp(rng.normal(0, 0.3, n))
        ddx = np.float32(rad * np.cos(ang))
        ddy = np.float32(rad * np.sin(ang))
        # squares of floats are exact in double, so the double fma is a double sum of exact squares
        d = ddx.astype(np.float64) * ddx.astype(np.float64) + ddy.astype(np.float64) * ddy.astype(np.float64)
        exact = d <= eps2
        q2 = _fmaf(ddx, ddx, np.float32(ddy * ddy))
        conv = q2 <= lo
        notconv = q2 >= hi
        assert not np.any(conv & notconv)
        assert np.all(exact[conv])
        assert not np.any(exact[notconv])
        # the undecided band is narrow: the double test runs rarely
        assert np.mean(~(conv | notconv)) < 1e-3
