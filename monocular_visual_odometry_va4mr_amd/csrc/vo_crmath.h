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
// gfx950 and on x86 -- so the same source gives the same bits on both.  The series multiply by
// double-double coefficient tables instead of dividing (round 4: no division inside any
// series step).  Cost: a few hundred flops per call, paid a handful of times per chain per
// frame (and per SIFT keypoint).
//
// The header is C and HIP C++ (the oracle in oracle/*.c includes it as well).
#pragma once

#ifdef __HIPCC__
#define VO_CR __host__ __device__ inline
#define VCR_TAB static __constant__ const
#else
#define VO_CR static inline
#define VCR_TAB static const
#endif

/* Series coefficients as double-doubles (hi, lo pairs; tools/gen_crmath_tables.py, 300-bit
 * mpmath): the nested series below multiply by them instead of dividing by integers, so no
 * evaluation step needs a division (a division is the longest dependent chain on both CPUs
 * and gfx950).  Index k holds the factor of nested term k. */
VCR_TAB double VCR_SIN_C[64] = {
    0x1.0000000000000p+0, 0x0.0p+0,
    0x1.5555555555555p-3, 0x1.5555555555555p-57,
    0x1.999999999999ap-5, -0x1.999999999999ap-59,
    0x1.8618618618618p-6, 0x1.8618618618618p-60,
    0x1.c71c71c71c71cp-7, 0x1.c71c71c71c71cp-61,
    0x1.29e4129e4129ep-7, 0x1.04a7904a7904ap-61,
    0x1.a41a41a41a41ap-8, 0x1.0690690690690p-62,
    0x1.3813813813814p-8, -0x1.fb1fb1fb1fb20p-62,
    0x1.e1e1e1e1e1e1ep-9, 0x1.e1e1e1e1e1e1ep-65,
    0x1.7f405fd017f40p-9, 0x1.7f405fd017f40p-63,
    0x1.3813813813814p-9, -0x1.fb1fb1fb1fb20p-63,
    0x1.03091b51f5e1ap-9, 0x1.3bb3194be3ab0p-63,
    0x1.b4e81b4e81b4fp-10, -0x1.f92c5f92c5f93p-64,
    0x1.756cac201756dp-10, -0x1.4f7fa2a4d4f80p-64,
    0x1.42d6625d51f87p-10, -0x1.064e2febd299ep-66,
    0x1.19e0119e0119ep-10, 0x1.19e0119e0119ep-70,
    0x1.f07c1f07c1f08p-11, -0x1.f07c1f07c1f08p-66,
    0x1.b89401b89401cp-11, -0x1.daff91daff91ep-65,
    0x1.899c0f601899cp-11, 0x1.ec0313381ec03p-68,
    0x1.61c544c0161c5p-11, 0x1.1300587151300p-65,
    0x1.3fb013fb013fbp-11, 0x1.3fb013fb013fbp-71,
    0x1.224dadc900489p-11, 0x1.b5b92009126d7p-66,
    0x1.08cabb37565e2p-11, 0x1.08cabb37565e2p-71,
    0x1.e500b5e044342p-12, -0x1.9b1d9a2b19d03p-66,
    0x1.bdd2b899406f7p-12, 0x1.2b899406f74aep-66,
    0x1.9b34ce68019b3p-12, 0x1.339a0066cd33ap-66,
    0x1.7c7862170949fp-12, 0x1.943fe83879de9p-70,
    0x1.610e4ef473283p-12, -0x1.4fd11c198388bp-66,
    0x1.4880522014880p-12, 0x1.4880522014880p-66,
    0x1.326c069552243p-12, 0x1.50f1c93d31d2dp-66,
    0x1.1e7f0550db594p-12, 0x1.1e7f0550db594p-72,
    0x1.0c73e00431cf8p-12, 0x1.0c73e00431cf8p-72,
};
VCR_TAB double VCR_COS_C[64] = {
    0x1.0000000000000p+0, 0x0.0p+0,
    0x1.0000000000000p-1, 0x0.0p+0,
    0x1.5555555555555p-4, 0x1.5555555555555p-58,
    0x1.1111111111111p-5, 0x1.1111111111111p-61,
    0x1.2492492492492p-6, 0x1.2492492492492p-60,
    0x1.6c16c16c16c17p-7, -0x1.f49f49f49f49fp-62,
    0x1.f07c1f07c1f08p-8, -0x1.f07c1f07c1f08p-63,
    0x1.6816816816817p-8, -0x1.fa5fa5fa5fa60p-62,
    0x1.1111111111111p-8, 0x1.1111111111111p-64,
    0x1.ac5701ac5701bp-9, -0x1.d47f29d47f29dp-64,
    0x1.58ed2308158edp-9, 0x1.1840ac7691841p-64,
    0x1.1bb4a4046ed29p-9, 0x1.1bb4a4046ed29p-69,
    0x1.dae6076b981dbp-10, -0x1.9f89467e251a0p-66,
    0x1.934c67f9b2ce6p-10, 0x1.934c67f9b2ce6p-70,
    0x1.5ac056b015ac0p-10, 0x1.5ac056b015ac0p-64,
    0x1.2d50a012d50a0p-10, 0x1.2d50a012d50a0p-66,
    0x1.0842108421084p-10, 0x1.0842108421084p-65,
    0x1.d347a4bc01d34p-11, 0x1.e92f0074d1e93p-65,
    0x1.a01a01a01a01ap-11, 0x1.a01a01a01a01ap-71,
    0x1.74e4b040174e5p-11, -0x1.3effa2c6d3f00p-65,
    0x1.5015015015015p-11, 0x1.5015015015015p-71,
    0x1.3076ee7525c2cp-11, 0x1.3076ee7525c2cp-71,
    0x1.151b9a3fdd5c9p-11, -0x1.a3fdd5c8cb804p-66,
    0x1.fa8ef6d92aca5p-12, 0x1.cd0c1eaba7f22p-67,
    0x1.d0cb58f6ec074p-12, 0x1.96b1edd80e866p-67,
    0x1.abfd7e03c2fa6p-12, -0x1.1de2532c833d4p-66,
    0x1.8b64018b64019p-12, -0x1.26ff9d26ff9d2p-66,
    0x1.6e60f6292563ap-12, 0x1.47bcbc32ce722p-66,
    0x1.54725e6bb82fep-12, 0x1.54725e6bb82fep-72,
    0x1.3d2c729a8f68ep-12, -0x1.cba76a15fdd4fp-66,
    0x1.2835399057efdp-12, -0x1.7492f2678e9bap-67,
    0x1.15411deb26da8p-12, 0x1.15411deb26da8p-72,
};
VCR_TAB double VCR_ASIN_C[122] = {
    0x1.0000000000000p+0, 0x0.0p+0,
    0x1.5555555555555p-3, 0x1.5555555555555p-57,
    0x1.ccccccccccccdp-2, -0x1.999999999999ap-57,
    0x1.30c30c30c30c3p-1, 0x1.8618618618618p-58,
    0x1.5c71c71c71c72p-1, -0x1.c71c71c71c71cp-56,
    0x1.7904a7904a790p-1, 0x1.29e4129e4129ep-55,
    0x1.8d20d20d20d21p-1, -0x1.6f96f96f96f97p-56,
    0x1.9c09c09c09c0ap-1, -0x1.fb1fb1fb1fb20p-56,
    0x1.a787878787878p-1, 0x1.e1e1e1e1e1e1ep-55,
    0x1.b0a7ac29eb0a8p-1, -0x1.4f5853d614f58p-55,
    0x1.b813813813814p-1, -0x1.fb1fb1fb1fb20p-55,
    0x1.be3ab0103091bp-1, 0x1.47d78693bb319p-55,
    0x1.c369d0369d037p-1, -0x1.8bf258bf258bfp-55,
    0x1.c7d7281d2c7d7p-1, 0x1.40e963eb940e9p-56,
    0x1.cbaa3f0ddf364p-1, -0x1.7f5e94ced1570p-55,
    0x1.cf008cf008cf0p-1, 0x1.19e0119e0119ep-58,
    0x1.d1f07c1f07c1fp-1, 0x1.f07c1f07c1f08p-59,
    0x1.d48b66d48b66dp-1, 0x1.22d9b522d9b52p-55,
    0x1.d6def164b56dfp-1, -0x1.d36952421d369p-58,
    0x1.d8f5fb29cd8f6p-1, -0x1.358c9c281358dp-59,
    0x1.dad949ad949aep-1, -0x1.ad949ad949ad9p-55,
    0x1.dc90048936b72p-1, 0x1.0048936b72401p-55,
    0x1.de20108cabb37p-1, 0x1.5978804232aedp-55,
    0x1.df8e53d55f700p-1, 0x1.e500b5e044342p-56,
    0x1.e0dee95c4ca03p-1, 0x1.ee95c4ca037bap-55,
    0x1.e215487baee21p-1, 0x1.521eebb885522p-55,
    0x1.e334639381ac0p-1, 0x1.db967a9ccb9c7p-55,
    0x1.e43ec00b08727p-1, 0x1.e8e6505581772p-55,
    0x1.e536894da2537p-1, -0x1.dac976b25dac9p-55,
    0x1.e61d9ff1a2efbp-1, 0x1.00264d80d2aa4p-57,
    0x1.e6f5a5e90ed41p-1, 0x1.8337ad2f4876ap-56,
    0x1.e7c008639f002p-1, 0x1.8e7c008639f00p-57,
    0x1.e87e07e07e07ep-1, 0x1.f81f81f81f820p-59,
    0x1.e930bed02e506p-1, -0x1.4e62e1512a42fp-55,
    0x1.e9d92710ce05bp-1, -0x1.af3ff2084b137p-56,
    0x1.ea781e7e4cda0p-1, -0x1.c055b608728e6p-56,
    0x1.eb0e6ac39ab0ep-1, 0x1.ab0e6ac39ab0ep-55,
    0x1.eb9cbc9048536p-1, 0x1.58a787b3fbf0ep-55,
    0x1.ec23b24ebe081p-1, -0x1.b35b841cb27b9p-56,
    0x1.eca3da7180353p-1, -0x1.46608ceba499ep-56,
    0x1.ed1db5698f7c8p-1, 0x1.8050e89cc2afcp-55,
    0x1.ed91b7547b129p-1, 0x1.333ae74004d09p-55,
    0x1.ee00496e00497p-1, -0x1.ffb691ffb6920p-57,
    0x1.ee69cb4ee69cbp-1, 0x1.3b9a72d3b9a73p-55,
    0x1.eece94010bc46p-1, 0x1.4657568dba718p-57,
    0x1.ef2ef2ef2ef2fp-1, -0x1.a21a21a21a21ap-58,
    0x1.ef8b30b5eab25p-1, 0x1.c4e0860b4007bp-56,
    0x1.efe38fda636b3p-1, -0x1.d65ffa7ef0765p-55,
    0x1.f0384d6a725d4p-1, 0x1.c26b5392ea01cp-60,
    0x1.f089a1897901fp-1, 0x1.ee5fbac32735cp-56,
    0x1.f0d7bfec88ab2p-1, 0x1.e508026eea9b8p-56,
    0x1.f122d848205c0p-1, 0x1.445fb6b437f26p-56,
    0x1.f16b16b16b16bp-1, 0x1.6b16b16b16b17p-57,
    0x1.f1b0a3f49fcd7p-1, 0x1.cccf1c7c0cd20p-58,
    0x1.f1f3a5e1e71f4p-1, -0x1.6878638316878p-55,
    0x1.f2343f91f7dd7p-1, 0x1.42613348ab6bep-56,
    0x1.f27291a3704dbp-1, -0x1.bfeb49776c6b7p-56,
    0x1.f2aeba71cdc6cp-1, -0x1.bce7ab54a15f3p-58,
    0x1.f2e8d646c586dp-1, 0x1.00d47735cba36p-55,
    0x1.f320ff86a781bp-1, 0x1.05a6d05817a0ap-56,
    0x1.f3574ed85da7bp-1, 0x1.19878bc7045f6p-55,
};
VCR_TAB double VCR_EXP_C[50] = {
    0x1.0000000000000p+0, 0x0.0p+0,
    0x1.0000000000000p+0, 0x0.0p+0,
    0x1.0000000000000p-1, 0x0.0p+0,
    0x1.5555555555555p-2, 0x1.5555555555555p-56,
    0x1.0000000000000p-2, 0x0.0p+0,
    0x1.999999999999ap-3, -0x1.999999999999ap-57,
    0x1.5555555555555p-3, 0x1.5555555555555p-57,
    0x1.2492492492492p-3, 0x1.2492492492492p-57,
    0x1.0000000000000p-3, 0x0.0p+0,
    0x1.c71c71c71c71cp-4, 0x1.c71c71c71c71cp-58,
    0x1.999999999999ap-4, -0x1.999999999999ap-58,
    0x1.745d1745d1746p-4, -0x1.745d1745d1746p-59,
    0x1.5555555555555p-4, 0x1.5555555555555p-58,
    0x1.3b13b13b13b14p-4, -0x1.3b13b13b13b14p-58,
    0x1.2492492492492p-4, 0x1.2492492492492p-58,
    0x1.1111111111111p-4, 0x1.1111111111111p-60,
    0x1.0000000000000p-4, 0x0.0p+0,
    0x1.e1e1e1e1e1e1ep-5, 0x1.e1e1e1e1e1e1ep-61,
    0x1.c71c71c71c71cp-5, 0x1.c71c71c71c71cp-59,
    0x1.af286bca1af28p-5, 0x1.af286bca1af28p-59,
    0x1.999999999999ap-5, -0x1.999999999999ap-59,
    0x1.8618618618618p-5, 0x1.8618618618618p-59,
    0x1.745d1745d1746p-5, -0x1.745d1745d1746p-60,
    0x1.642c8590b2164p-5, 0x1.642c8590b2164p-60,
    0x1.5555555555555p-5, 0x1.5555555555555p-59,
};
VCR_TAB double VCR_LOG_C[46] = {
    0x1.0000000000000p+0, 0x0.0p+0,
    0x1.5555555555555p-2, 0x1.5555555555555p-56,
    0x1.3333333333333p-1, 0x1.999999999999ap-56,
    0x1.6db6db6db6db7p-1, -0x1.2492492492492p-56,
    0x1.8e38e38e38e39p-1, -0x1.c71c71c71c71cp-57,
    0x1.a2e8ba2e8ba2fp-1, -0x1.d1745d1745d17p-55,
    0x1.b13b13b13b13bp-1, 0x1.3b13b13b13b14p-57,
    0x1.bbbbbbbbbbbbcp-1, -0x1.1111111111111p-55,
    0x1.c3c3c3c3c3c3cp-1, 0x1.e1e1e1e1e1e1ep-56,
    0x1.ca1af286bca1bp-1, -0x1.af286bca1af28p-58,
    0x1.cf3cf3cf3cf3dp-1, -0x1.8618618618618p-58,
    0x1.d37a6f4de9bd3p-1, 0x1.e9bd37a6f4deap-55,
    0x1.d70a3d70a3d71p-1, -0x1.70a3d70a3d70ap-55,
    0x1.da12f684bda13p-1, -0x1.2f684bda12f68p-58,
    0x1.dcb08d3dcb08dp-1, 0x1.ee58469ee5847p-56,
    0x1.def7bdef7bdefp-1, 0x1.ef7bdef7bdef8p-55,
    0x1.e0f83e0f83e10p-1, -0x1.f07c1f07c1f08p-55,
    0x1.e2be2be2be2bep-1, 0x1.5f15f15f15f16p-56,
    0x1.e45306eb3e453p-1, 0x1.bacf914c1bad0p-59,
    0x1.e5be5be5be5bep-1, 0x1.6f96f96f96f97p-55,
    0x1.e7063e7063e70p-1, 0x1.8f9c18f9c18fap-55,
    0x1.e82fa0be82fa1p-1, -0x1.05f417d05f418p-55,
    0x1.e93e93e93e93fp-1, -0x1.b05b05b05b05bp-55,
};

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
VO_CR vcr_dd vcr_tab(const double* t, int k) { return vcr_mk(t[2 * k], t[2 * k + 1]); }
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
        t = t * r2 * VCR_COS_C[2 * n];                      /* r^2n / (2n)! */
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
        p = vcr_mul(vcr_mul(r2, p), vcr_tab(VCR_SIN_C, k));
        p = vcr_add_d(vcr_neg(p), 1.0);
    }
    return vcr_mul(r, p);
}
VO_CR vcr_dd vcr_cos_red(vcr_dd r)
{
    const vcr_dd r2 = vcr_mul(r, r);
    vcr_dd p = vcr_mk(1.0, 0.0);
    for (int k = vcr_trig_terms(r2.hi); k >= 1; --k) {      /* p = 1 - r^2 p / ((2k-1)(2k)) */
        p = vcr_mul(vcr_mul(r2, p), vcr_tab(VCR_COS_C, k));
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
    for (int k = n; k >= 1; --k)                           /* p = 1 + s^2 p (2k-1)^2 / ((2k)(2k+1)) */
        p = vcr_add_d(vcr_mul(vcr_mul(s2, p), vcr_tab(VCR_ASIN_C, k)), 1.0);
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
    for (int k = 24; k >= 1; --k) p = vcr_add_d(vcr_mul(vcr_mul(x, p), vcr_tab(VCR_EXP_C, k)), 1.0);
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
    /* terms 1..n with u^(2(n+1)) < 7.7e-34 (the tail is below 2^-110 of p; at most 22, the
       count |u| < 0.172 needs): near x = 1, the RANSAC update's usual input, a third of them */
    int n = 1;
    double t = u2.hi;
    while (n < 22) {
        t *= u2.hi;
        if (t < 7.7e-34) break;
        ++n;
    }
    vcr_dd p = vcr_mk(1.0, 0.0);                           /* 1 + u^2/3 + u^4/5 + ... */
    for (int k = n; k >= 1; --k)                           /* p = 1 + u^2 p (2k-1) / (2k+1) */
        p = vcr_add_d(vcr_mul(vcr_mul(u2, p), vcr_tab(VCR_LOG_C, k)), 1.0);
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
