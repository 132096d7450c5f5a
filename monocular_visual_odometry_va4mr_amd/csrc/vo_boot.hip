// Bootstrap geometry for gfx950 (VisualOdometryPipeLine.py:293-323): findEssentialMat
// RANSAC with the 5-point minimal solver (one thread per hypothesis, wave-parallel
// Sampson scoring, OpenCV's sequential update rule), recoverPose (4-way cheirality by
// DLT triangulation), and the bootstrap assembly into chain state.  Mirrors
// oracle/vo_oracle_geom.c (vo_o_five_point / vo_o_find_essential / vo_o_recover_pose).
#include "vo_dgeom.h"

namespace {

using namespace vg;

// ------------------------------------------------------------------ 5-point
struct MonoTab { int e[20][3]; int prod[20][20]; };

constexpr MonoTab make_mono()
{
    MonoTab t{};
    const int M[20][3] = {
        {3, 0, 0}, {0, 3, 0}, {2, 1, 0}, {1, 2, 0}, {2, 0, 1}, {2, 0, 0}, {0, 2, 1}, {0, 2, 0},
        {1, 1, 1}, {1, 1, 0}, {1, 0, 2}, {1, 0, 1}, {1, 0, 0}, {0, 1, 2}, {0, 1, 1}, {0, 1, 0},
        {0, 0, 3}, {0, 0, 2}, {0, 0, 1}, {0, 0, 0}};
    for (int i = 0; i < 20; ++i)
        for (int k = 0; k < 3; ++k) t.e[i][k] = M[i][k];
    for (int i = 0; i < 20; ++i)
        for (int j = 0; j < 20; ++j) {
            int a = M[i][0] + M[j][0], b = M[i][1] + M[j][1], c = M[i][2] + M[j][2];
            t.prod[i][j] = -1;
            if (a + b + c > 3) continue;
            for (int k = 0; k < 20; ++k)
                if (M[k][0] == a && M[k][1] == b && M[k][2] == c) t.prod[i][j] = k;
        }
    return t;
}

constexpr MonoTab MTc = make_mono();

struct Poly3 { double c[20]; };

VO_DEV void p_zero(Poly3& p) { for (int i = 0; i < 20; ++i) p.c[i] = 0.0; }
VO_DEV void p_axpy(double s, const Poly3& a, Poly3& y) { for (int i = 0; i < 20; ++i) y.c[i] += s * a.c[i]; }

// The oracle's p_mul (oracle/vo_oracle_geom.c) over the operands' structural supports only
// (D = 1: the linear polynomials of the null space, monomials x, y, z, 1; D = 2: their products,
// every monomial of degree <= 2), fully
// unrolled with the product table resolved at compile time, so no array is indexed at run time
// (the loop over all 20 x 20 index pairs kept its operands in scratch memory; k_essential 2.59 ->
// 2.15 ms per call at 32 chains).  Every entry outside a support is exactly zero, which p_mul
// skips, and the supports are visited in ascending order: the same additions in the same order.
template <int DA, int DB>
VO_DEV void p_mul_s(const Poly3& a, const Poly3& b, Poly3& out)
{
    constexpr int S1[4] = {12, 15, 18, 19};
    constexpr int S2[10] = {5, 7, 9, 11, 12, 14, 15, 17, 18, 19};
    constexpr int NA = DA == 1 ? 4 : 10, NB = DB == 1 ? 4 : 10;
    Poly3 r;
#pragma unroll
    for (int k = 0; k < 20; ++k) r.c[k] = 0.0;
#pragma unroll
    for (int ii = 0; ii < NA; ++ii) {
        const int i = DA == 1 ? S1[ii] : S2[ii];
        const double ai = a.c[i];
#pragma unroll
        for (int jj = 0; jj < NB; ++jj) {
            const int j = DB == 1 ? S1[jj] : S2[jj];
            const int k = MTc.prod[i][j];
            if (k < 0) continue;
            const double bj = b.c[j];
            if (ai != 0.0 && bj != 0.0) r.c[k] += ai * bj;
        }
    }
    out = r;
}

VO_DEV int gauss_solve(double* A, int n, double* B, int m)
{
    for (int c = 0; c < n; ++c) {
        int p = c;
        double best = fabs(A[c * n + c]);
        for (int r = c + 1; r < n; ++r) if (fabs(A[r * n + c]) > best) { best = fabs(A[r * n + c]); p = r; }
        if (best == 0.0) return 0;
        if (p != c) {
            for (int k = 0; k < n; ++k) { double t = A[c * n + k]; A[c * n + k] = A[p * n + k]; A[p * n + k] = t; }
            for (int k = 0; k < m; ++k) { double t = B[c * m + k]; B[c * m + k] = B[p * m + k]; B[p * m + k] = t; }
        }
        double inv = 1.0 / A[c * n + c];
        for (int r = c + 1; r < n; ++r) {
            double f = A[r * n + c] * inv;
            if (f == 0.0) continue;
            for (int k = c; k < n; ++k) A[r * n + k] -= f * A[c * n + k];
            for (int k = 0; k < m; ++k) B[r * m + k] -= f * B[c * m + k];
        }
    }
    for (int c = n - 1; c >= 0; --c) {
        double inv = 1.0 / A[c * n + c];
        for (int k = 0; k < m; ++k) {
            double s = B[c * m + k];
            for (int j = c + 1; j < n; ++j) s -= A[c * n + j] * B[j * m + k];
            B[c * m + k] = s * inv;
        }
    }
    return 1;
}

struct Cplx { double re, im; };
VO_DEV Cplx c_mul(Cplx a, Cplx b) { return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }
VO_DEV Cplx c_sub(Cplx a, Cplx b) { return {a.re - b.re, a.im - b.im}; }
VO_DEV Cplx c_add(Cplx a, Cplx b) { return {a.re + b.re, a.im + b.im}; }
VO_DEV Cplx c_div(Cplx a, Cplx b)
{
    double t = 1. / (b.re * b.re + b.im * b.im);
    return {(a.re * b.re + a.im * b.im) * t, (-a.re * b.im + a.im * b.re) * t};
}

// The sweep of solve_poly at degree 10 (the five-point polynomial's usual degree) with every loop
// unrolled, so the roots and coefficients stay in registers: the runtime-bound loops indexed them
// dynamically, which put both arrays in scratch memory (about 200 scratch loads per sweep, 300
// sweeps per solve; the sweeps almost never reach maxDiff == 0).  Same operations, same order.
VO_DEV void solve_poly10(const Cplx (&co)[11], Cplx (&roots)[10])
{
    for (int iter = 0; iter < 300; ++iter) {
        double maxDiff = 0;
#pragma unroll
        for (int i = 0; i < 10; ++i) {
            const Cplx p = roots[i];
            Cplx num = co[10], denom = co[10];
#pragma unroll
            for (int j = 0; j < 10; ++j) {
                num = c_add(c_mul(num, p), co[10 - j - 1]);
                if (j != i) {
                    Cplx d = c_sub(p, roots[j]);
                    if (!(d.re == 0 && d.im == 0)) denom = c_mul(denom, d);
                }
            }
            num = c_div(num, denom);
            roots[i] = c_sub(p, num);
            double a = sqrt(num.re * num.re + num.im * num.im);
            if (a > maxDiff) maxDiff = a;
        }
        if (maxDiff <= 0) break;
    }
}

// cv::solvePoly (Weierstrass iteration, 300 sweeps max)
VO_DEV int solve_poly(const double* c_in, int n0, Cplx* roots)
{
    if (n0 == 10 && fabs(c_in[10]) + fabs(0.0) > DBL_EPSILON) {
        Cplx co[11], r[10];
#pragma unroll
        for (int i = 0; i <= 10; ++i) { co[i].re = c_in[i]; co[i].im = 0; }
        Cplx p = {1, 0}, rr = {1, 1};
#pragma unroll
        for (int i = 0; i < 10; ++i) { r[i] = p; p = c_mul(p, rr); }
        solve_poly10(co, r);
#pragma unroll
        for (int i = 0; i < 10; ++i) {
            if (fabs(r[i].im) < 1e-100) r[i].im = 0;
            roots[i] = r[i];
        }
        return 10;
    }

    Cplx co[11];
    for (int i = 0; i <= n0; ++i) { co[i].re = c_in[i]; co[i].im = 0; }
    int n = n0;
    for (; n > 1; --n) if (fabs(co[n].re) + fabs(co[n].im) > DBL_EPSILON) break;
    Cplx p = {1, 0}, r = {1, 1};
    for (int i = 0; i < n; ++i) { roots[i] = p; p = c_mul(p, r); }
    for (int iter = 0; iter < 300; ++iter) {
        double maxDiff = 0;
        for (int i = 0; i < n; ++i) {
            p = roots[i];
            Cplx num = co[n], denom = co[n];
            for (int j = 0; j < n; ++j) {
                num = c_add(c_mul(num, p), co[n - j - 1]);
                if (j != i) {
                    Cplx d = c_sub(p, roots[j]);
                    if (!(d.re == 0 && d.im == 0)) denom = c_mul(denom, d);
                }
            }
            num = c_div(num, denom);
            roots[i] = c_sub(p, num);
            double a = sqrt(num.re * num.re + num.im * num.im);
            if (a > maxDiff) maxDiff = a;
        }
        if (maxDiff <= 0) break;
    }
    for (int i = 0; i < n; ++i) if (fabs(roots[i].im) < 1e-100) roots[i].im = 0;
    return n;
}

// five_point in three parts: the Groebner-basis coefficients of the degree-10 polynomial in z
// (false if the 10x10 elimination is singular), the roots, and each real root's essential matrix.
VO_DEV bool five_point_coeffs(const double* q1, const double* q2, double (&basis)[4][9], double (&b)[3][13],
                              double (&coeffs)[11])
{
    double Qt[9 * 5];
    for (int i = 0; i < 5; ++i) {
        double x1 = q1[2 * i], y1 = q1[2 * i + 1], x2 = q2[2 * i], y2 = q2[2 * i + 1];
        double row[9] = {x1 * x2, y1 * x2, x2, x1 * y2, y1 * y2, y2, x1, y1, 1.0};
        for (int j = 0; j < 9; ++j) Qt[j * 5 + i] = row[j];
    }
    double H[5][9], hn[5];
    for (int k = 0; k < 5; ++k) {
        double nrm = 0;
        for (int i = k; i < 9; ++i) nrm += Qt[i * 5 + k] * Qt[i * 5 + k];
        nrm = sqrt(nrm);
        double alpha = Qt[k * 5 + k] > 0 ? -nrm : nrm;
        for (int i = 0; i < 9; ++i) H[k][i] = (i < k) ? 0.0 : Qt[i * 5 + k];
        H[k][k] -= alpha;
        double vn = 0;
        for (int i = k; i < 9; ++i) vn += H[k][i] * H[k][i];
        hn[k] = vn;
        if (vn == 0) continue;
        for (int j = k; j < 5; ++j) {
            double s = 0;
            for (int i = k; i < 9; ++i) s += H[k][i] * Qt[i * 5 + j];
            s = 2.0 * s / vn;
            for (int i = k; i < 9; ++i) Qt[i * 5 + j] -= s * H[k][i];
        }
    }
    for (int b = 0; b < 4; ++b) {
        double v[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        v[5 + b] = 1.0;
        for (int k = 4; k >= 0; --k) {
            if (hn[k] == 0) continue;
            double s = 0;
            for (int i = k; i < 9; ++i) s += H[k][i] * v[i];
            s = 2.0 * s / hn[k];
            for (int i = k; i < 9; ++i) v[i] -= s * H[k][i];
        }
        for (int i = 0; i < 9; ++i) basis[b][i] = v[i];
    }
    Poly3 Ep[9];
    for (int e = 0; e < 9; ++e) {
        p_zero(Ep[e]);
        Ep[e].c[12] = basis[0][e];
        Ep[e].c[15] = basis[1][e];
        Ep[e].c[18] = basis[2][e];
        Ep[e].c[19] = basis[3][e];
    }
    double A[100], Bm[100];
    {
        Poly3 t1, acc;
        p_zero(acc);
        const int cof[3][4] = {{4, 8, 5, 7}, {3, 8, 5, 6}, {3, 7, 4, 6}};
        const double sg[3] = {1, -1, 1};
        #pragma unroll
        for (int c = 0; c < 3; ++c) {
            Poly3 m1, m2;
            p_mul_s<1, 1>(Ep[cof[c][0]], Ep[cof[c][1]], m1);
            p_mul_s<1, 1>(Ep[cof[c][2]], Ep[cof[c][3]], m2);
            p_axpy(-1.0, m2, m1);
            p_mul_s<1, 2>(Ep[c], m1, t1);
            p_axpy(sg[c], t1, acc);
        }
        for (int c = 0; c < 20; ++c) { if (c < 10) A[c] = acc.c[c]; else Bm[c - 10] = acc.c[c]; }
    }
    {
        Poly3 EEt[9];
        #pragma unroll
        for (int i = 0; i < 3; ++i)
            #pragma unroll
            for (int j = 0; j < 3; ++j) {
                p_zero(EEt[i * 3 + j]);
                #pragma unroll
                for (int k = 0; k < 3; ++k) {
                    Poly3 m;
                    p_mul_s<1, 1>(Ep[i * 3 + k], Ep[j * 3 + k], m);
                    p_axpy(1.0, m, EEt[i * 3 + j]);
                }
            }
        Poly3 tr;
        p_zero(tr);
        p_axpy(1.0, EEt[0], tr);
        p_axpy(1.0, EEt[4], tr);
        p_axpy(1.0, EEt[8], tr);
        #pragma unroll
        for (int i = 0; i < 3; ++i)
            #pragma unroll
            for (int j = 0; j < 3; ++j) {
                Poly3 acc, m;
                p_zero(acc);
                #pragma unroll
                for (int k = 0; k < 3; ++k) {
                    p_mul_s<2, 1>(EEt[i * 3 + k], Ep[k * 3 + j], m);
                    p_axpy(2.0, m, acc);
                }
                p_mul_s<2, 1>(tr, Ep[i * 3 + j], m);
                p_axpy(-1.0, m, acc);
                const int r = 1 + i * 3 + j;
                for (int c = 0; c < 20; ++c) { if (c < 10) A[r * 10 + c] = acc.c[c]; else Bm[r * 10 + (c - 10)] = acc.c[c]; }
            }
    }
    if (!gauss_solve(A, 10, Bm, 10)) return false;
    for (int i = 0; i < 3; ++i) {
        const double* g1 = Bm + (4 + 2 * i) * 10;
        const double* g2 = Bm + (5 + 2 * i) * 10;
        double r1[13], r2[13];
        for (int k = 0; k < 13; ++k) { r1[k] = 0; r2[k] = 0; }
        r1[1] = g1[0]; r1[2] = g1[1]; r1[3] = g1[2];
        r1[5] = g1[3]; r1[6] = g1[4]; r1[7] = g1[5];
        r1[9] = g1[6]; r1[10] = g1[7]; r1[11] = g1[8]; r1[12] = g1[9];
        r2[0] = g2[0]; r2[1] = g2[1]; r2[2] = g2[2];
        r2[4] = g2[3]; r2[5] = g2[4]; r2[6] = g2[5];
        r2[8] = g2[6]; r2[9] = g2[7]; r2[10] = g2[8]; r2[11] = g2[9];
        for (int k = 0; k < 13; ++k) b[i][k] = r1[k] - r2[k];
    }
    double P[3][3][5];
    for (int i = 0; i < 3; ++i) {
        for (int k = 0; k < 5; ++k) P[i][0][k] = P[i][1][k] = P[i][2][k] = 0;
        for (int k = 0; k < 4; ++k) { P[i][0][3 - k] = b[i][k]; P[i][1][3 - k] = b[i][4 + k]; }
        for (int k = 0; k < 5; ++k) P[i][2][4 - k] = b[i][8 + k];
    }
    for (int k = 0; k < 11; ++k) coeffs[k] = 0;
    {
        const int perm[6][3] = {{0, 1, 2}, {0, 2, 1}, {1, 0, 2}, {1, 2, 0}, {2, 0, 1}, {2, 1, 0}};
        const double psign[6] = {1, -1, -1, 1, 1, -1};
        for (int s = 0; s < 6; ++s) {
            double t1[9], t2[11];
            for (int k = 0; k < 9; ++k) t1[k] = 0;
            for (int k = 0; k < 11; ++k) t2[k] = 0;
            for (int a = 0; a < 5; ++a) for (int c = 0; c < 5; ++c)
                if (a + c < 9) t1[a + c] += P[0][perm[s][0]][a] * P[1][perm[s][1]][c];
            for (int a = 0; a < 9; ++a) for (int c = 0; c < 5; ++c)
                if (a + c < 11) t2[a + c] += t1[a] * P[2][perm[s][2]][c];
            for (int k = 0; k < 11; ++k) coeffs[k] += psign[s] * t2[k];
        }
    }
    return true;
}

// the essential matrix of one root (false: complex, or no finite (x, y)), normalised
VO_DEV bool five_point_root_E(const Cplx root, const double (&basis)[4][9], const double (&b)[3][13], double* E)
{
    {
        if (fabs(root.im) > 1e-10) return false;
        double z1 = root.re, z2 = z1 * z1, z3 = z2 * z1, z4 = z3 * z1;
        double Bz[9];
        for (int j = 0; j < 3; ++j) {
            const double* br = b[j];
            Bz[j * 3 + 0] = br[0] * z3 + br[1] * z2 + br[2] * z1 + br[3];
            Bz[j * 3 + 1] = br[4] * z3 + br[5] * z2 + br[6] * z1 + br[7];
            Bz[j * 3 + 2] = br[8] * z4 + br[9] * z3 + br[10] * z2 + br[11] * z1 + br[12];
        }
        double Aw[9], w[3], V[9];
        for (int q = 0; q < 9; ++q) Aw[q] = Bz[q];
        svd_jacobi<3, 3>(Aw, w, V);
        double xy1[3] = {V[2], V[5], V[8]};
        if (fabs(xy1[2]) < 1e-10) return false;
        double x = xy1[0] / xy1[2], y = xy1[1] / xy1[2];
        double ev[9], nrm = 0;
        for (int e = 0; e < 9; ++e) {
            ev[e] = basis[0][e] * x + basis[1][e] * y + basis[2][e] * z1 + basis[3][e];
            nrm += ev[e] * ev[e];
        }
        nrm = sqrt(nrm);
        for (int e = 0; e < 9; ++e) E[e] = ev[e] / nrm;
    }
    return true;
}

VO_DEV int five_point(const double* q1, const double* q2, double* E10)
{
    double basis[4][9], b[3][13], coeffs[11];
    if (!five_point_coeffs(q1, q2, basis, b, coeffs)) return 0;
    Cplx roots[10];
    const int nroots = solve_poly(coeffs, 10, roots);
    int count = 0;
    for (int i = 0; i < nroots; ++i)
        if (five_point_root_E(roots[i], basis, b, E10 + count * 9)) ++count;
    return count;
}

// five_point for one hypothesis on 10 lanes (li = 0..9 of a group starting at lane gb): the
// coefficients on every lane, then the degree-10 Weierstrass sweeps with lane li owning root li,
// pipelined (root t's update needs the new roots 0..t-1 only in its denominator, whose factors
// are multiplied in j order: lane i takes factor t (new root t) at step t < i and its old-root
// factors t+1..9 at step i; its numerator, which depends on its own root only, at the sweep's
// start), then each real root's essential matrix on its lane, written in root order.  The same
// operations in the same order as five_point, so the same models.  Other degrees: lane 0 runs
// five_point.
VO_DEV int five_point_grp(const double* q1, const double* q2, double* E10, int li, int gb)
{
    double basis[4][9], b[3][13], coeffs[11];
    if (!five_point_coeffs(q1, q2, basis, b, coeffs)) return 0;
    if (!(fabs(coeffs[10]) + fabs(0.0) > DBL_EPSILON)) {
        int nm = 0;
        if (li == 0) nm = five_point(q1, q2, E10);
        return __shfl(nm, gb, 64);
    }
    Cplx co[11], r[10];
#pragma unroll
    for (int i = 0; i <= 10; ++i) { co[i].re = coeffs[i]; co[i].im = 0; }
    {
        Cplx p = {1, 0}, rr = {1, 1};
#pragma unroll
        for (int i = 0; i < 10; ++i) { r[i] = p; p = c_mul(p, rr); }
    }
    for (int iter = 0; iter < 300; ++iter) {
        Cplx pm = r[0];
#pragma unroll
        for (int i = 1; i < 10; ++i) if (li == i) pm = r[i];
        Cplx num = co[10], den = co[10];
#pragma unroll
        for (int j = 0; j < 10; ++j) num = c_add(c_mul(num, pm), co[10 - j - 1]);
        double maxDiff = 0;
#pragma unroll
        for (int t = 0; t < 10; ++t) {
            Cplx nr = {0, 0};
            double a = 0;
            if (li == t) {
#pragma unroll
                for (int j = t + 1; j < 10; ++j) {
                    Cplx d = c_sub(pm, r[j]);
                    if (!(d.re == 0 && d.im == 0)) den = c_mul(den, d);
                }
                const Cplx q = c_div(num, den);
                nr = c_sub(pm, q);
                a = sqrt(q.re * q.re + q.im * q.im);
            }
            r[t].re = __shfl(nr.re, gb + t, 64);
            r[t].im = __shfl(nr.im, gb + t, 64);
            a = __shfl(a, gb + t, 64);
            if (a > maxDiff) maxDiff = a;
            if (li > t) {
                Cplx d = c_sub(pm, r[t]);
                if (!(d.re == 0 && d.im == 0)) den = c_mul(den, d);
            }
        }
        if (maxDiff <= 0) break;
    }
    Cplx mine = r[0];
#pragma unroll
    for (int i = 1; i < 10; ++i) if (li == i) mine = r[i];
    if (fabs(mine.im) < 1e-100) mine.im = 0;
    double E[9];
    const bool ok = five_point_root_E(mine, basis, b, E);
    const uint64_t m = (__ballot(ok) >> gb) & 0x3FFull;
    if (ok) {
        const int slot = __popcll(m & ((1ull << li) - 1ull));
        for (int e = 0; e < 9; ++e) E10[slot * 9 + e] = E[e];
    }
    return __popcll(m);
}

// ------------------------------------------------------------------ E-RANSAC
#define EHYP 64

struct EssArgs {
    double K[9];
    double prob, threshold;
    int max_iters;
    const float* p0;
    const float* p1;
    const int32_t* counts;
    int cap;
    double* work;            // [B][work_stride]: q1 (2cap), q2 (2cap), models (EHYP*90)
    int64_t work_stride;
    double* E;               // [B][9]
    uint8_t* mask;           // [B][cap]
    int32_t* ok;             // [B]
    const int32_t* chain_status;
};

// WPE 2: the build for more chains than CUs (at most 256 registers per lane, two blocks per CU;
// 768-chain bootstrap 0.365 vs 0.368-0.404 s).  Scoring is in the sequential rule's order, one
// hypothesis per wave per batch, and stops at the running adaptive count (identical result to
// scoring all EHYP).  Measured and not kept: the five-point solves spread over 16 lanes of each
// wave instead of one whole wave (0.376 s).
template <int WPE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, 8))) k_essential(EssArgs A)
{
    __shared__ int sub[EHYP][5];
    __shared__ int nmod[EHYP];
    __shared__ int cnt[EHYP][10];
    __shared__ double bestE[9];
    __shared__ int sh[4];
    const int b = blockIdx.x, tid = threadIdx.x;
    if (A.chain_status && A.chain_status[b] != 0) return;
    const int n = A.counts[b];
    const float* p0 = A.p0 + (int64_t)b * A.cap * 2;
    const float* p1 = A.p1 + (int64_t)b * A.cap * 2;
    uint8_t* mask = A.mask + (int64_t)b * A.cap;
    double* q1 = A.work + (int64_t)b * A.work_stride;
    double* q2 = q1 + 2 * A.cap;
    double* models = q2 + 2 * A.cap;
    const double fx = A.K[0], fy = A.K[4], cx = A.K[2], cy = A.K[5];
    for (int i = tid; i < n; i += blockDim.x) {
        q1[2 * i] = ((double)p0[2 * i] - cx) / fx;
        q1[2 * i + 1] = ((double)p0[2 * i + 1] - cy) / fy;
        q2[2 * i] = ((double)p1[2 * i] - cx) / fx;
        q2[2 * i + 1] = ((double)p1[2 * i + 1] - cy) / fy;
    }
    double thr_d = A.threshold / ((fx + fy) / 2);
    const float thr = (float)(thr_d * thr_d);
    __syncthreads();
    if (n < 5) {
        for (int i = tid; i < n; i += blockDim.x) mask[i] = 0;
        if (tid == 0) A.ok[b] = 0;
        return;
    }
    if (n == 5) {
        if (tid == 0) {
            double E10[90];
            int nm = five_point(q1, q2, E10);
            A.ok[b] = nm > 0;
            for (int q = 0; q < 9; ++q) A.E[9 * b + q] = nm > 0 ? E10[q] : 0.0;
            for (int i = 0; i < 5; ++i) mask[i] = nm > 0 ? 1 : 0;
        }
        return;
    }
    uint64_t rng = ~0ULL;
    double lnum = 0.0;      // thread 0: log(1 - prob), formed at the first improvement
    bool have_lnum = false;
    if (tid == 0) { sh[0] = 0; sh[1] = A.max_iters > 1 ? A.max_iters : 1; sh[2] = 0; }
    __syncthreads();
    // one block per CU (WPE 1): each hypothesis on 10 lanes (five_point_grp), 6 per wave, 24 per
    // round; more chains than CUs (WPE 2): one hypothesis per lane of wave 0, 64 per round
    constexpr int NH = WPE == 1 ? 24 : EHYP;
    while (true) {
        const int it0 = sh[0], niters0 = sh[1];
        if (it0 >= niters0) break;
        if (tid == 0) {
            for (int h = 0; h < NH; ++h)
                for (int i = 0; i < 5; ++i) {
                    for (;;) {
                        int v = (int)(rng_next(rng) % (uint32_t)n);
                        int j;
                        for (j = 0; j < i; ++j) if (v == sub[h][j]) break;
                        sub[h][i] = v;
                        if (j == i) break;
                    }
                }
        }
        __syncthreads();
        if constexpr (WPE == 1) {
            const int lane = lane_id(), g = lane / 10, li = lane - 10 * g;
            const int h = wave_id() * 6 + g;
            if (lane < 60 && h < NH) {
                int nm = 0;
                if (it0 + h < niters0) {
                    double s1[10], s2[10];
                    for (int j = 0; j < 5; ++j) {
                        const int id = sub[h][j];
                        s1[2 * j] = q1[2 * id]; s1[2 * j + 1] = q1[2 * id + 1];
                        s2[2 * j] = q2[2 * id]; s2[2 * j + 1] = q2[2 * id + 1];
                    }
                    nm = five_point_grp(s1, s2, models + 90 * h, li, 10 * g);
                }
                if (li == 0) nmod[h] = nm;
            }
        } else if (tid < EHYP) {
            const int h = tid;
            int nm = 0;
            if (it0 + h < niters0) {
                double s1[10], s2[10];
                for (int j = 0; j < 5; ++j) {
                    const int id = sub[h][j];
                    s1[2 * j] = q1[2 * id]; s1[2 * j + 1] = q1[2 * id + 1];
                    s2[2 * j] = q2[2 * id]; s2[2 * j + 1] = q2[2 * id + 1];
                }
                nm = five_point(s1, s2, models + 90 * h);
            }
            nmod[h] = nm;
        }
        __syncthreads();
        {
            const int w = wave_id(), lane = lane_id(), nw = blockDim.x >> 6;
            for (int h0 = 0; h0 < NH; h0 += nw) {
                if (it0 + h0 >= sh[1]) break;                                 // block-uniform
                const int h = h0 + w;
                if (h < NH)
                    for (int m = 0; m < nmod[h]; ++m) {
                        const double* Em = models + 90 * h + 9 * m;
                        int c = 0;
                        for (int i = lane; i < n; i += 64)
                            c += sampson_err(Em, q1[2 * i], q1[2 * i + 1], q2[2 * i], q2[2 * i + 1]) <= thr;
                        c = wave_sum_i32(c);
                        if (lane == 0) cnt[h][m] = c;
                    }
                __syncthreads();
                if (tid == 0) {
                    int niters = sh[1], best = sh[2];
                    const int h1 = h0 + nw < NH ? h0 + nw : NH;
                    for (int hh = h0; hh < h1; ++hh) {
                        if (it0 + hh >= niters) break;
                        for (int m = 0; m < nmod[hh]; ++m) {
                            const int good = cnt[hh][m];
                            if (good > (best > 4 ? best : 4)) {
                                best = good;
                                for (int q = 0; q < 9; ++q) bestE[q] = models[90 * hh + 9 * m + q];
                                if (!have_lnum) { lnum = ransac_log_num(A.prob); have_lnum = true; }
                                niters = ransac_update_niters_ln(lnum, (double)(n - good) / n, 5, niters);
                            }
                        }
                    }
                    sh[1] = niters;
                    sh[2] = best;
                }
                __syncthreads();
            }
        }
        if (tid == 0) sh[0] = it0 + NH;
        __syncthreads();
    }
    const bool ok = sh[2] > 0;
    for (int i = tid; i < n; i += blockDim.x)
        mask[i] = ok ? (sampson_err(bestE, q1[2 * i], q1[2 * i + 1], q2[2 * i], q2[2 * i + 1]) <= thr) : 0;
    if (tid == 0) {
        A.ok[b] = ok;
        for (int q = 0; q < 9; ++q) A.E[9 * b + q] = ok ? bestE[q] : 0.0;
    }
}

// ------------------------------------------------------------------ recoverPose
struct RecArgs {
    double K[9];
    const double* E;
    const float* p0;
    const float* p1;
    const int32_t* counts;
    int cap;
    double* R;               // [B][9]
    double* t;               // [B][3]
    uint8_t* mask;           // [B][cap] (may be null)
    int32_t* n_good;         // [B]
    const int32_t* chain_status;
    int sign_fix;            // apply t *= sign(t_z) (VisualOdometryPipeLine.py:317)
};

// recoverPose's two rotations and translation from E (thread 0; the block's shared copies)
VO_DEV void rp_decompose(const double* E, double* R1, double* R2, double* tt)
{
    double U[9], w[3], V[9];
    for (int q = 0; q < 9; ++q) U[q] = E[q];
    svd_jacobi<3, 3>(U, w, V);
    if (det3(U) < 0) for (int i = 0; i < 9; ++i) U[i] = -U[i];
    if (det3(V) < 0) for (int i = 0; i < 9; ++i) V[i] = -V[i];
    const double W[9] = {0, 1, 0, -1, 0, 0, 0, 0, 1}, Wt[9] = {0, -1, 0, 1, 0, 0, 0, 0, 1};
    double Vt[9], UW[9];
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) Vt[i * 3 + j] = V[j * 3 + i];
    matmul3(U, W, UW);
    matmul3(UW, Vt, R1);
    matmul3(U, Wt, UW);
    matmul3(UW, Vt, R2);
    for (int i = 0; i < 3; ++i) tt[i] = U[i * 3 + 2];
}

// the four-way cheirality test of points i0, i0 + stride, ... (< n): per-candidate counts in g,
// per-point bits in mask (if non-null)
VO_DEV void rp_count(const RecArgs& A, const double* R1, const double* R2, const double* tt, int n, int i0,
                     int stride, int (&g)[4], uint8_t* mask)
{
    const int b = blockIdx.x;
    const float* p0 = A.p0 + (int64_t)b * A.cap * 2;
    const float* p1 = A.p1 + (int64_t)b * A.cap * 2;
    const double fx = A.K[0], fy = A.K[4], cx = A.K[2], cy = A.K[5];
    const double dist = 50.0;
    const double P0[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    for (int i = i0; i < n; i += stride) {
        const double x1 = ((double)p0[2 * i] - cx) / fx, y1 = ((double)p0[2 * i + 1] - cy) / fy;
        const double x2 = ((double)p1[2 * i] - cx) / fx, y2 = ((double)p1[2 * i + 1] - cy) / fy;
        uint8_t bits = 0;
        for (int c = 0; c < 4; ++c) {
            const double* Rc = (c == 0 || c == 2) ? R1 : R2;
            const double sg = (c < 2) ? 1.0 : -1.0;
            double P[12];
            for (int r = 0; r < 3; ++r) {
                for (int q = 0; q < 3; ++q) P[r * 4 + q] = Rc[r * 3 + q];
                P[r * 4 + 3] = sg * tt[r];
            }
            double Q[4];
            tri_one(P0, P, x1, y1, x2, y2, Q);
            double X = Q[0], Y = Q[1], Z = Q[2], Wh = Q[3];
            int m = (Z * Wh) > 0;
            X /= Wh; Y /= Wh; Z /= Wh;
            const double W1 = Wh / Wh;
            m = m && (Z < dist);
            const double z2 = P[8] * X + P[9] * Y + P[10] * Z + P[11] * W1;
            m = m && (z2 > 0);
            m = m && (z2 < dist);
            g[c] += m;
            bits |= (uint8_t)(m << c);
        }
        if (mask) mask[i] = bits;
    }
}

// the candidate with the most points in front of both cameras (first of equals), its R and t
VO_DEV void rp_pick(const RecArgs& A, const int* good, const double* R1, const double* R2, const double* tt, int& sel)
{
    const int b = blockIdx.x;
    if (good[0] >= good[1] && good[0] >= good[2] && good[0] >= good[3]) sel = 0;
    else if (good[1] >= good[0] && good[1] >= good[2] && good[1] >= good[3]) sel = 1;
    else if (good[2] >= good[0] && good[2] >= good[1] && good[2] >= good[3]) sel = 2;
    else sel = 3;
    if (threadIdx.x == 0) {
        const double* Rs = (sel == 0 || sel == 2) ? R1 : R2;
        double t3[3];
        for (int i = 0; i < 3; ++i) t3[i] = (sel < 2) ? tt[i] : -tt[i];
        if (A.sign_fix) {
            const double s = (t3[2] > 0) ? 1.0 : ((t3[2] < 0) ? -1.0 : 0.0);   // np.sign
            for (int i = 0; i < 3; ++i) t3[i] *= s;
        }
        for (int q = 0; q < 9; ++q) A.R[9 * b + q] = Rs[q];
        for (int q = 0; q < 3; ++q) A.t[3 * b + q] = t3[q];
        A.n_good[b] = good[sel];
    }
}

__global__ void __launch_bounds__(256) k_recover_pose(RecArgs A)
{
    __shared__ double R1[9], R2[9], tt[3];
    __shared__ int lds[16];
    __shared__ int good[4];
    const int b = blockIdx.x, tid = threadIdx.x;
    if (A.chain_status && A.chain_status[b] != 0) return;
    const int n = A.counts[b];
    if (tid == 0) rp_decompose(A.E + 9 * b, R1, R2, tt);
    __syncthreads();
    int g[4] = {0, 0, 0, 0};
    uint8_t* mask = A.mask ? A.mask + (int64_t)b * A.cap : nullptr;
    rp_count(A, R1, R2, tt, n, tid, blockDim.x, g, mask);
    for (int c = 0; c < 4; ++c) {
        const int s = block_sum_i32(g[c], lds);
        if (tid == 0) good[c] = s;
    }
    __syncthreads();
    int sel;
    rp_pick(A, good, R1, R2, tt, sel);
    if (mask)
        for (int i = tid; i < n; i += blockDim.x) mask[i] = (mask[i] >> sel) & 1;
}

// The bootstrap's recoverPose (no mask output) with few chains: the cheirality counts over
// RP_SPLIT blocks per chain (integer sums, order-free) into gcount [B][4] (zeroed by
// k_boot_apply), then the pick by one block per chain.  One block per chain left most CUs idle
// while each thread triangulated ~12 points four ways.
#define RP_SPLIT 8
__global__ void __launch_bounds__(256) k_recover_count(RecArgs A, int32_t* gcount)
{
    __shared__ double R1[9], R2[9], tt[3];
    __shared__ int lds[16];
    const int b = blockIdx.x, tid = threadIdx.x;
    if (A.chain_status && A.chain_status[b] != 0) return;
    const int n = A.counts[b];
    if (tid == 0) rp_decompose(A.E + 9 * b, R1, R2, tt);
    __syncthreads();
    int g[4] = {0, 0, 0, 0};
    rp_count(A, R1, R2, tt, n, blockIdx.y * blockDim.x + tid, gridDim.y * blockDim.x, g, nullptr);
    for (int c = 0; c < 4; ++c) {
        const int s = block_sum_i32(g[c], lds);
        if (tid == 0 && s) atomicAdd(&gcount[4 * b + c], s);
    }
}
__global__ void __launch_bounds__(64) k_recover_pick(RecArgs A, const int32_t* gcount)
{
    __shared__ double R1[9], R2[9], tt[3];
    const int b = blockIdx.x;
    if (A.chain_status && A.chain_status[b] != 0) return;
    if (threadIdx.x == 0) rp_decompose(A.E + 9 * b, R1, R2, tt);
    __syncthreads();
    const int good[4] = {gcount[4 * b], gcount[4 * b + 1], gcount[4 * b + 2], gcount[4 * b + 3]};
    int sel;
    rp_pick(A, good, R1, R2, tt, sel);
}

// ------------------------------------------------------------------ bootstrap assembly
// initialization :306-313: candidates <- matches, E-inlier split, filter_potential
__global__ void __launch_bounds__(256) k_boot_apply(vo_dims d, vo_state s, const float* pts0, const float* pts1,
                                                    const int32_t* counts, int cap, const uint8_t* emask,
                                                    const int32_t* eok, int32_t* gcount)
{
    __shared__ int lds[16];
    const int b = blockIdx.x, tid = threadIdx.x;
    const int n = counts[b];
    if (tid < 4) gcount[4 * b + tid] = 0;                              // k_recover_count's sums
    if (tid == 0) {
        s.status[b] = 0;
        s.nL[b] = 0;
        s.nC[b] = 0;
        s.nF[b] = 1;
        double* R0 = s.pose_R + (int64_t)b * d.fcap * 9;
        double* t0 = s.pose_t + (int64_t)b * d.fcap * 3;
        for (int q = 0; q < 9; ++q) R0[q] = (q % 4 == 0) ? 1.0 : 0.0;       // transforms[0] = (I, 0)
        for (int q = 0; q < 3; ++q) t0[q] = 0.0;
        if (n == 0) s.status[b] = VO_ST_NO_MATCHES;
        else if (!eok[b]) s.status[b] = VO_ST_ESSENTIAL_FAILED;
        else if (n > d.pcap) s.status[b] = VO_ST_CAPACITY;
    }
    __syncthreads();
    if (s.status[b] != 0) return;
    const float* a0 = pts0 + (int64_t)b * cap * 2;
    const float* a1 = pts1 + (int64_t)b * cap * 2;
    const uint8_t* m = emask + (int64_t)b * cap;
    const int kcap = d.ncap > d.pcap ? d.ncap : d.pcap;
    float* ck = s.c_kp + (int64_t)b * d.pcap * 2;
    float* cf = s.c_first + (int64_t)b * d.pcap * 2;
    int32_t* ct = s.c_tau + (int64_t)b * d.pcap;
    float* inl = s.inl_kp + (int64_t)b * kcap * 2;
    float* outl = s.outl_kp + (int64_t)b * kcap * 2;
    int nin = 0, nout = 0;
    for (int base = 0; base < n; base += blockDim.x) {
        const int i = base + tid;
        const bool valid = i < n;
        const bool in = valid && m[i] == 1;
        int tin, tout;
        const int pin = nin + block_scan_flag(in, lds, &tin);
        const int pout = nout + block_scan_flag(valid && !in, lds, &tout);
        if (in) {
            ck[2 * pin] = a1[2 * i]; ck[2 * pin + 1] = a1[2 * i + 1];
            cf[2 * pin] = a0[2 * i]; cf[2 * pin + 1] = a0[2 * i + 1];
            ct[pin] = 0;                                                // len(transforms) - 1
            inl[2 * pin] = a1[2 * i]; inl[2 * pin + 1] = a1[2 * i + 1];
        } else if (valid) {
            outl[2 * pout] = a1[2 * i]; outl[2 * pout + 1] = a1[2 * i + 1];
        }
        nin += tin;
        nout += tout;
    }
    if (tid == 0) {
        s.nC[b] = nin;
        s.nInl[b] = nin;
        s.nOutl[b] = nout;
    }
}

// :315-317 pose into slot 1 (written by k_recover_pose into pose arrays directly)
__global__ void k_boot_finish(vo_dims d, vo_state s)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= d.B || s.status[b] != 0) return;
    s.num_pts[(int64_t)b * d.fcap + 1] = s.nInl[b];                      // num_pts = [sum(inliers)]
    s.nF[b] = 2;
}

__global__ void k_copy_pose(vo_dims d, vo_state s, const double* R, const double* t)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= d.B || s.status[b] != 0) return;
    for (int q = 0; q < 9; ++q) s.pose_R[((int64_t)b * d.fcap + 1) * 9 + q] = R[9 * b + q];
    for (int q = 0; q < 3; ++q) s.pose_t[((int64_t)b * d.fcap + 1) * 3 + q] = t[3 * b + q];
}

}  // namespace

// ======================================================================= host side
#define VO_STREAM(s) ((hipStream_t)(s))
static inline int hip_rc() { return hipGetLastError() == hipSuccess ? VO_OK : VO_EHIP; }

static void fill_ess(EssArgs& A, const vo_opts* o, const float* p0, const float* p1, const int32_t* counts, int cap,
                     double prob, double thr, int iters, double* E, uint8_t* mask, int32_t* ok, double* work,
                     int64_t ws, const int32_t* st)
{
    for (int i = 0; i < 9; ++i) A.K[i] = o->K[i];
    A.prob = prob; A.threshold = thr; A.max_iters = iters;
    A.p0 = p0; A.p1 = p1; A.counts = counts; A.cap = cap;
    A.work = work; A.work_stride = ws; A.E = E; A.mask = mask; A.ok = ok; A.chain_status = st;
}

static void launch_essential(const EssArgs& A, int B, hipStream_t st)
{
    const int n_cu = device_cus() > 0 ? device_cus() : 256;          // of the current device
    if (B > n_cu) hipLaunchKernelGGL(k_essential<2>, dim3(B), dim3(256), 0, st, A);
    else hipLaunchKernelGGL(k_essential<1>, dim3(B), dim3(256), 0, st, A);
}

extern "C" int vo_find_essential(const vo_opts* o, int B, const float* p0, const float* p1, const int32_t* counts,
                                 int32_t cap, double prob, double threshold, int32_t max_iters, double* E,
                                 uint8_t* mask, int32_t* ok, double* work, int32_t work_doubles, vo_stream_t stream)
{
    if (!o || B < 1 || !p0 || !p1 || !counts || !E || !mask || !ok || !work) return VO_EARG;
    if ((int64_t)work_doubles < 4LL * cap + 90 * EHYP) return VO_EARG;
    EssArgs A;
    fill_ess(A, o, p0, p1, counts, cap, prob, threshold, max_iters, E, mask, ok, work, work_doubles, nullptr);
    launch_essential(A, B, VO_STREAM(stream));
    return hip_rc();
}

extern "C" int vo_recover_pose(const vo_opts* o, int B, const double* E, const float* p0, const float* p1,
                               const int32_t* counts, int32_t cap, double* R, double* t, uint8_t* mask,
                               int32_t* n_good, vo_stream_t stream)
{
    if (!o || B < 1 || !E || !p0 || !p1 || !counts || !R || !t || !n_good) return VO_EARG;
    RecArgs A;
    for (int i = 0; i < 9; ++i) A.K[i] = o->K[i];
    A.E = E; A.p0 = p0; A.p1 = p1; A.counts = counts; A.cap = cap; A.R = R; A.t = t; A.mask = mask;
    A.n_good = n_good; A.chain_status = nullptr; A.sign_fix = 0;
    hipLaunchKernelGGL(k_recover_pose, dim3(B), dim3(256), 0, VO_STREAM(stream), A);
    return hip_rc();
}

extern "C" int vo_triangulate(const vo_dims* d, const vo_opts* o, const vo_state* s, int force, vo_stream_t stream);

extern "C" int vo_bootstrap(const vo_dims* d, const vo_opts* o, const vo_state* s, const float* pts0,
                            const float* pts1, const int32_t* counts, int32_t cap, vo_stream_t stream)
{
    if (!d || !o || !s || !pts0 || !pts1 || !counts) return VO_EARG;
    if (d->work_stride < 4LL * cap + 90 * EHYP + 16) return VO_EARG;
    hipStream_t st = VO_STREAM(stream);
    // scratch: q1/q2/models in each chain's fp64 work region; E/R/t ([B][9], [B][9], [B][3])
    // in trk_pts (free outside the tracking stage); E-mask / ok / n_good in the PnP buffers
    EssArgs A;
    fill_ess(A, o, pts0, pts1, counts, cap, 0.99, 1.0, 1000, nullptr, s->pnp_mask, s->pnp_ok, s->work,
             d->work_stride, nullptr);
    double* Ebuf = (double*)s->trk_pts;
    double* Rbuf = Ebuf + 9 * (int64_t)d->B;
    double* tbuf = Rbuf + 9 * (int64_t)d->B;
    int32_t* gcount = (int32_t*)(tbuf + 3 * (int64_t)d->B);                // [B][4]
    A.E = Ebuf;
    if (cap > d->ncap) return VO_EARG;            // the E mask lives in pnp_mask [B][ncap]
    A.mask = s->pnp_mask;
    A.cap = cap;
    launch_essential(A, d->B, st);
    hipLaunchKernelGGL(k_boot_apply, dim3(d->B), dim3(256), 0, st, *d, *s, pts0, pts1, counts, cap,
                       (const uint8_t*)s->pnp_mask, (const int32_t*)s->pnp_ok, gcount);
    RecArgs Rg;
    for (int i = 0; i < 9; ++i) Rg.K[i] = o->K[i];
    Rg.E = Ebuf; Rg.p0 = s->c_first; Rg.p1 = s->c_kp; Rg.counts = s->nC; Rg.cap = d->pcap;
    Rg.R = Rbuf; Rg.t = tbuf; Rg.mask = nullptr; Rg.n_good = s->pnp_ninl; Rg.chain_status = s->status;
    Rg.sign_fix = 1;
    if (d->B >= (device_cus() > 0 ? device_cus() : 256)) {
        hipLaunchKernelGGL(k_recover_pose, dim3(d->B), dim3(256), 0, st, Rg);
    } else {
        hipLaunchKernelGGL(k_recover_count, dim3(d->B, RP_SPLIT), dim3(256), 0, st, Rg, gcount);
        hipLaunchKernelGGL(k_recover_pick, dim3(d->B), dim3(64), 0, st, Rg, (const int32_t*)gcount);
    }
    hipLaunchKernelGGL(k_copy_pose, dim3((d->B + 63) / 64), dim3(64), 0, st, *d, *s, (const double*)Rbuf,
                       (const double*)tbuf);
    int rc = vo_triangulate(d, o, s, 1, stream);
    if (rc) return rc;
    hipLaunchKernelGGL(k_boot_finish, dim3((d->B + 63) / 64), dim3(64), 0, st, *d, *s);
    return hip_rc();
}
