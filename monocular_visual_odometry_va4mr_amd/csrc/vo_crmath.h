// Correctly rounded double cos / sin / acos / exp2 / log / integer power for the libm calls
// of the path whose results feed decisions or poses:
//   * Rodrigues (both directions) inside solvePnPRansac and after it
//     (VisualOdometryPipeLine.py:343,354);
//   * RANSACUpdateNumIters (pow, log) of solvePnPRansac / findEssentialMat (:308,:343);
//   * the SIFT keypoint size (pow(2, .)) and descriptor rotation (cos, sin) (:226-227).
//
// Neither libm is exact: OCML (device) is faithful to 1-2 ulp and glibc 2.35 (host, the
// oracle) misrounds too (acos by up to 1 ulp on ~0.06 % of inputs, measured against
// mpmath).  With each side calling its own libm the GPU pose differed from the oracle's by
// one ulp on about 1 step in 36 (malaga_c3 frame 12, |dR| 7e-18).  So the oracle and the
// kernels both call these functions instead, and tests/test_crmath.py checks them against
// 200-bit mpmath values: the results are the correctly rounded ones (OpenCV-level parity of
// those ulps stays unpinned, as for every other OpenCV arithmetic detail).
//
// Each function evaluates f(x) in double-double (hi + lo, ~2^-100 relative) with exact
// fma-based products and rounds once, so the result is RN(f(x)) unless f(x) lies within
// ~2^-100 of a rounding midpoint.  Only + - * / sqrt fma are used -- all correctly rounded on
// gfx950 and on x86 -- so the same source gives the same bits on both.  Cost: a few hundred
// flops per call, paid a handful of times per chain per frame.
//
// The header is C and HIP C++ (the oracle in oracle/*.c includes it as well).
#pragma once

#ifdef __HIPCC__
#define VO_CR __host__ __device__ inline
#else
#define VO_CR static inline
#endif

typedef struct { double hi, lo; } vcr_dd;

VO_CR vcr_dd vcr_mk(double hi, double lo)
{
    vcr_dd r;
    r.hi = hi;
    r.lo = lo;
    return r;
}

VO_CR vcr_dd vcr_two_sum(double a, double b)
{
    const double s = a + b, bb = s - a;
    return vcr_mk(s, (a - (s - bb)) + (b - bb));
}
VO_CR vcr_dd vcr_fast_two_sum(double a, double b)          /* |a| >= |b| or a == 0 */
{
    const double s = a + b;
    return vcr_mk(s, b - (s - a));
}
VO_CR vcr_dd vcr_two_prod(double a, double b)
{
    const double p = a * b;
    return vcr_mk(p, __builtin_fma(a, b, -p));
}
VO_CR vcr_dd vcr_add(vcr_dd x, vcr_dd y)
{
    vcr_dd s = vcr_two_sum(x.hi, y.hi), t = vcr_two_sum(x.lo, y.lo);
    s.lo += t.hi;
    s = vcr_fast_two_sum(s.hi, s.lo);
    s.lo += t.lo;
    return vcr_fast_two_sum(s.hi, s.lo);
}
VO_CR vcr_dd vcr_add_d(vcr_dd x, double y)
{
    vcr_dd s = vcr_two_sum(x.hi, y);
    s.lo += x.lo;
    return vcr_fast_two_sum(s.hi, s.lo);
}
VO_CR vcr_dd vcr_mul(vcr_dd x, vcr_dd y)
{
    vcr_dd p = vcr_two_prod(x.hi, y.hi);
    p.lo += x.hi * y.lo + x.lo * y.hi;
    return vcr_fast_two_sum(p.hi, p.lo);
}
VO_CR vcr_dd vcr_mul_d(vcr_dd x, double y)
{
    vcr_dd p = vcr_two_prod(x.hi, y);
    p.lo += x.lo * y;
    return vcr_fast_two_sum(p.hi, p.lo);
}
VO_CR vcr_dd vcr_div_d(vcr_dd x, double y)                 /* y nonzero */
{
    const double q1 = x.hi / y;
    const vcr_dd r = vcr_two_prod(q1, y);                  /* q1 * y exactly */
    const double rem = ((x.hi - r.hi) - r.lo) + x.lo;
    return vcr_fast_two_sum(q1, rem / y);
}
VO_CR vcr_dd vcr_div(vcr_dd x, vcr_dd y)
{
    const double q1 = x.hi / y.hi;
    const vcr_dd r = vcr_add(x, vcr_mul_d(y, -q1));        /* x - q1 * y */
    const double q2 = r.hi / y.hi;
    const vcr_dd r2 = vcr_add(r, vcr_mul_d(y, -q2));
    return vcr_add_d(vcr_fast_two_sum(q1, q2), r2.hi / y.hi);
}
VO_CR vcr_dd vcr_neg(vcr_dd x) { return vcr_mk(-x.hi, -x.lo); }
VO_CR double vcr_round(vcr_dd x) { return x.hi + x.lo; }

/* pi/2 as three doubles; pi and ln 2 as double-doubles */
#define VCR_PIO2_1 1.5707963267948966192e+00
#define VCR_PIO2_2 6.1232339957367658e-17
#define VCR_PIO2_3 -1.4973849048591698e-33
#define VCR_PI_HI 3.141592653589793116e+00
#define VCR_PI_LO 1.2246467991473532e-16
#define VCR_LN2_HI 6.93147180559945286227e-01
#define VCR_LN2_LO 2.31904681384629955842e-17

/* number of nested Taylor terms of sin / cos for |r| <= pi/4 (term < 2^-110) */
VO_CR int vcr_trig_terms(double r2)
{
    double t = 1.0;
    int n = 1;
    while (n < 30) {
        t = t * r2 / ((2.0 * n - 1.0) * (2.0 * n));
        if (t < 7.7e-34) break;
        ++n;
    }
    return n + 1;
}
VO_CR vcr_dd vcr_sin_red(vcr_dd r)
{
    const vcr_dd r2 = vcr_mul(r, r);
    vcr_dd p = vcr_mk(1.0, 0.0);
    for (int k = vcr_trig_terms(r2.hi); k >= 1; --k) {      /* p = 1 - r^2 p / ((2k)(2k+1)) */
        p = vcr_div_d(vcr_mul(r2, p), (2.0 * k) * (2.0 * k + 1.0));
        p = vcr_add_d(vcr_neg(p), 1.0);
    }
    return vcr_mul(r, p);
}
VO_CR vcr_dd vcr_cos_red(vcr_dd r)
{
    const vcr_dd r2 = vcr_mul(r, r);
    vcr_dd p = vcr_mk(1.0, 0.0);
    for (int k = vcr_trig_terms(r2.hi); k >= 1; --k) {      /* p = 1 - r^2 p / ((2k-1)(2k)) */
        p = vcr_div_d(vcr_mul(r2, p), (2.0 * k - 1.0) * (2.0 * k));
        p = vcr_add_d(vcr_neg(p), 1.0);
    }
    return p;
}
/* x = q pi/2 + r with |r| <= pi/4 (Cody-Waite in double-double; |x| < 2^30) */
VO_CR vcr_dd vcr_reduce(double x, int* q)
{
    const double k = __builtin_rint(x * 0.63661977236758134308);
    *q = (int)((long long)k & 3);
    const vcr_dd a = vcr_two_prod(k, VCR_PIO2_1);
    vcr_dd r = vcr_two_sum(x, -a.hi);
    r = vcr_add_d(r, -a.lo);
    r = vcr_add(r, vcr_neg(vcr_two_prod(k, VCR_PIO2_2)));
    return vcr_add_d(r, -k * VCR_PIO2_3);
}

VO_CR double vcr_sin(double x)
{
    if (x == 0.0 || !(x - x == 0.0)) return x == 0.0 ? x : x - x;
    int q;
    const vcr_dd r = vcr_reduce(x, &q);
    vcr_dd v = (q & 1) ? vcr_cos_red(r) : vcr_sin_red(r);
    if (q & 2) v = vcr_neg(v);
    return vcr_round(v);
}
VO_CR double vcr_cos(double x)
{
    if (!(x - x == 0.0)) return x - x;
    int q;
    const vcr_dd r = vcr_reduce(x, &q);
    vcr_dd v = (q & 1) ? vcr_sin_red(r) : vcr_cos_red(r);
    if (((q + 1) >> 1) & 1) v = vcr_neg(v);               /* q = 1, 2 */
    return vcr_round(v);
}

/* asin(s), |s| <= 1/2: s (1 + a1 s^2 (1 + a2 s^2 (...))), a_k = (2k-1)^2 / ((2k)(2k+1)) */
VO_CR vcr_dd vcr_asin_small(vcr_dd s)
{
    const vcr_dd s2 = vcr_mul(s, s);
    int n = 1;
    double t = 1.0;
    while (n < 60) {
        t *= s2.hi;
        if (t < 7.7e-34) break;
        ++n;
    }
    vcr_dd p = vcr_mk(1.0, 0.0);
    for (int k = n; k >= 1; --k) {
        const double num = (2.0 * k - 1.0) * (2.0 * k - 1.0);
        p = vcr_div_d(vcr_mul_d(vcr_mul(s2, p), num), (2.0 * k) * (2.0 * k + 1.0));
        p = vcr_add_d(p, 1.0);
    }
    return vcr_mul(s, p);
}
VO_CR vcr_dd vcr_sqrt_dd(double h)
{
    const double s0 = __builtin_sqrt(h);
    if (s0 == 0.0) return vcr_mk(0.0, 0.0);
    const double e = __builtin_fma(-s0, s0, h);            /* h - s0^2 exactly */
    return vcr_fast_two_sum(s0, e / (2.0 * s0));
}
VO_CR double vcr_acos(double c)
{
    if (!(c >= -1.0 && c <= 1.0)) return (c - c) / (c - c);     /* NaN */
    if (c >= 0.5) {                        /* 2 asin(sqrt((1-c)/2)); 1-c exact (Sterbenz) */
        const vcr_dd a = vcr_asin_small(vcr_sqrt_dd((1.0 - c) * 0.5));
        return vcr_round(vcr_mul_d(a, 2.0));
    }
    if (c > -0.5) {                        /* pi/2 - asin(c) */
        const vcr_dd a = vcr_asin_small(vcr_mk(c, 0.0));
        return vcr_round(vcr_add(vcr_mk(VCR_PIO2_1, VCR_PIO2_2), vcr_neg(a)));
    }
    const vcr_dd a = vcr_asin_small(vcr_sqrt_dd((1.0 + c) * 0.5));   /* pi - 2 asin(.) */
    return vcr_round(vcr_add(vcr_mk(VCR_PI_HI, VCR_PI_LO), vcr_neg(vcr_mul_d(a, 2.0))));
}

/* exp(x) of a double-double |x| <= 0.36 (nested Taylor 1 + x/1 (1 + x/2 (...))) */
VO_CR vcr_dd vcr_exp_red(vcr_dd x)
{
    vcr_dd p = vcr_mk(1.0, 0.0);
    for (int k = 24; k >= 1; --k) p = vcr_add_d(vcr_div_d(vcr_mul(x, p), (double)k), 1.0);
    return p;
}
/* 2^y, finite y with |y| < 1000 */
VO_CR double vcr_exp2(double y)
{
    if (!(y - y == 0.0)) return y > 0 ? y : 0.0;
    const double n = __builtin_rint(y);
    const double f = y - n;                                /* exact, |f| <= 1/2 */
    const vcr_dd p = vcr_exp_red(vcr_mul_d(vcr_mk(VCR_LN2_HI, VCR_LN2_LO), f));
    return __builtin_ldexp(vcr_round(p), (int)n);
}

/* natural log of a positive normal double: x = 2^e m, m in [sqrt(1/2), sqrt(2)),
   log x = e ln2 + 2 atanh(u), u = (m-1)/(m+1) (|u| < 0.172), atanh by nested series */
VO_CR double vcr_log(double x)
{
    if (!(x > 0.0)) return x == 0.0 ? -1.0 / 0.0 : (x - x) / (x - x);
    if (!(x - x == 0.0)) return x;
    int e;
    double m = __builtin_frexp(x, &e);                     /* m in [1/2, 1) */
    if (m < 0.70710678118654752440) { m *= 2.0; e -= 1; }
    const vcr_dd num = vcr_mk(m - 1.0, 0.0);               /* exact (Sterbenz) */
    const vcr_dd u = vcr_div(num, vcr_two_sum(m, 1.0));
    const vcr_dd u2 = vcr_mul(u, u);
    vcr_dd p = vcr_mk(1.0, 0.0);                           /* 1 + u^2/3 + u^4/5 + ... */
    for (int k = 22; k >= 1; --k)
        p = vcr_add_d(vcr_div_d(vcr_mul_d(vcr_mul(u2, p), 2.0 * k - 1.0), 2.0 * k + 1.0), 1.0);
    vcr_dd r = vcr_mul_d(vcr_mul(u, p), 2.0);
    r = vcr_add(r, vcr_mul_d(vcr_mk(VCR_LN2_HI, VCR_LN2_LO), (double)e));
    return vcr_round(r);
}

/* b^n for an integer n >= 0 (square-and-multiply in double-double) */
VO_CR double vcr_powi(double b, int n)
{
    vcr_dd r = vcr_mk(1.0, 0.0), p = vcr_mk(b, 0.0);
    while (n > 0) {
        if (n & 1) r = vcr_mul(r, p);
        n >>= 1;
        if (n) p = vcr_mul(p, p);
    }
    return vcr_round(r);
}
