"""vo_crmath.h (shared by the kernels and the C oracle) returns correctly rounded results.

The header is compiled here as C with gcc (the oracle's compiler) and checked against
200-bit mpmath values on inputs drawn from the ranges the path uses: Rodrigues angles and
cosines, RANSAC inlier ratios, SIFT keypoint-size exponents and descriptor angles.  The
same source runs on the GPU (only + - * / sqrt fma, all correctly rounded on gfx950), so
this pins the device results too; tests/test_gpu_parity.py checks GPU == oracle."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

mpmath = pytest.importorskip("mpmath")

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(REPO, "monocular_visual_odometry_va4mr_amd", "csrc")

SRC = r"""
#include "vo_crmath.h"
void crm_eval(int fn, const double* x, double* y, int n)
{
    for (int i = 0; i < n; ++i) {
        switch (fn) {
        case 0: y[i] = vcr_cos(x[i]); break;
        case 1: y[i] = vcr_sin(x[i]); break;
        case 2: y[i] = vcr_acos(x[i]); break;
        case 3: y[i] = vcr_exp2(x[i]); break;
        case 4: y[i] = vcr_log(x[i]); break;
        default: y[i] = vcr_powi(x[i], fn - 10); break;
        }
    }
}
"""


@pytest.fixture(scope="module")
def crm(tmp_path_factory):
    d = tmp_path_factory.mktemp("crm")
    c = d / "crm.c"
    c.write_text(SRC)
    so = d / "crm.so"
    subprocess.run(["gcc", "-O2", "-std=gnu11", "-fPIC", "-shared", "-ffp-contract=off", "-I", HDR,
                    str(c), "-o", str(so), "-lm"], check=True)
    lib = ctypes.CDLL(str(so))

    def ev(fn, x):
        x = np.ascontiguousarray(x, np.float64)
        y = np.empty_like(x)
        lib.crm_eval(fn, x.ctypes.data_as(ctypes.c_void_p), y.ctypes.data_as(ctypes.c_void_p), len(x))
        return y
    return ev


def _rn(f, xs):
    mpmath.mp.prec = 200
    return np.array([float(f(mpmath.mpf(float(x)))) for x in xs])


def test_trig_correctly_rounded(crm):
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(-np.pi, np.pi, 1500), rng.uniform(-1e-3, 1e-3, 500),
                        rng.uniform(-7, 7, 500), [0.0, 1e-300, np.pi / 4, np.pi / 2, np.pi]])
    assert np.array_equal(crm(0, x), _rn(mpmath.cos, x))
    assert np.array_equal(crm(1, x), _rn(mpmath.sin, x))


def test_acos_correctly_rounded(crm):
    rng = np.random.default_rng(1)
    c = np.concatenate([rng.uniform(-1, 1, 2000), 1 - rng.uniform(0, 1e-6, 500), -1 + rng.uniform(0, 1e-6, 200),
                        [1.0, -1.0, 0.5, -0.5, 0.0, np.nextafter(0.5, 0), np.nextafter(-0.5, 0)]])
    assert np.array_equal(crm(2, c), _rn(mpmath.acos, c))
    assert np.isnan(crm(2, np.array([1.5, np.nan]))).all()


def test_exp2_log_powi_correctly_rounded(crm):
    rng = np.random.default_rng(2)
    y = np.concatenate([rng.uniform(-0.5, 2.5, 1500), [0.0, 1.0, 1 / 3, 2 / 3]])
    assert np.array_equal(crm(3, y), _rn(lambda v: mpmath.power(2, v), y))
    # the series length adapts to |u| = |m - 1| / (m + 1): inputs near 1 (few terms) and near
    # sqrt(1/2) 2^k (the full 22) are both covered
    x = np.concatenate([rng.uniform(1e-12, 1, 1500), rng.uniform(0.9, 1.1, 500), 1 - rng.uniform(0, 1e-6, 300),
                        np.sqrt(0.5) * 2.0 ** rng.integers(-20, 20, 200) * (1 + rng.uniform(-1e-3, 1e-3, 200)),
                        [0.01, 1.0, 2.0, 1e-300]])
    assert np.array_equal(crm(4, x), _rn(mpmath.log, x))
    for n in (4, 5):
        b = rng.uniform(0, 1, 800)
        assert np.array_equal(crm(10 + n, b), _rn(lambda v: v ** n, b))
