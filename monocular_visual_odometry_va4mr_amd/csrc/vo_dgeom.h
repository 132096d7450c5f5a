// fp64 geometry for gfx950 device code: one-sided Jacobi SVD, least squares, real
// polynomial roots (bracketed Newton, +-*/sqrt only), Gao P3P with Horn alignment,
// Rodrigues, Sampson error.  Each routine follows the operation order of its CPU
// oracle counterpart in oracle/vo_oracle_geom.c (which restates OpenCV 4.6, SURVEY.md
// Appendix A) so that, compiled with -ffp-contract=off, results agree bit for bit
// (the libm transcendentals acos/sin/cos/log/pow come from vo_crmath.h on both sides).
#pragma once
#include "vo_dev.h"
#include "vo_crmath.h"

#include <float.h>

namespace vg {

// (small M, N only: every loop is unrolled so A, w, V live in registers; the 12x12 EPnP
// decomposition uses svd_jacobi_wave below)
template <int M, int N>
VO_DEV void svd_jacobi(double* A, double* w, double* V)
{
    static_assert(N <= 6, "use svd_jacobi_wave for large matrices");
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
        for (int j = 0; j < N; ++j) V[i * N + j] = (i == j) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 60; ++sweep) {
        bool changed = false;
#pragma unroll
        for (int i = 0; i < N - 1; ++i) {
#pragma unroll
            for (int j = i + 1; j < N; ++j) {
                double alpha = 0, beta = 0, gamma = 0;
#pragma unroll
                for (int k = 0; k < M; ++k) {
                    double ai = A[k * N + i], aj = A[k * N + j];
                    alpha += ai * ai;
                    beta += aj * aj;
                    gamma += ai * aj;
                }
                if (alpha == 0.0 || beta == 0.0) continue;
                if (fabs(gamma) <= DBL_EPSILON * sqrt(alpha * beta)) continue;
                changed = true;
                double zeta = (beta - alpha) / (2.0 * gamma);
                double t = 1.0 / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                if (zeta < 0) t = -t;
                double c = 1.0 / sqrt(1.0 + t * t);
                double s = c * t;
#pragma unroll
                for (int k = 0; k < M; ++k) {
                    double ai = A[k * N + i], aj = A[k * N + j];
                    A[k * N + i] = c * ai - s * aj;
                    A[k * N + j] = s * ai + c * aj;
                }
#pragma unroll
                for (int k = 0; k < N; ++k) {
                    double vi = V[k * N + i], vj = V[k * N + j];
                    V[k * N + i] = c * vi - s * vj;
                    V[k * N + j] = s * vi + c * vj;
                }
            }
        }
        if (!changed) break;
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {
        double s = 0;
#pragma unroll
        for (int k = 0; k < M; ++k) s += A[k * N + i] * A[k * N + i];
        w[i] = sqrt(s);
    }
#pragma unroll
    for (int i = 0; i < N - 1; ++i) {
        // selection of the largest remaining w, then a swap, written with constant indices
        int b = i;
        double wb = w[i];
#pragma unroll
        for (int j = i + 1; j < N; ++j) if (w[j] > wb) { b = j; wb = w[j]; }
#pragma unroll
        for (int j = i + 1; j < N; ++j) {
            if (b == j) {
                double tw = w[i]; w[i] = w[j]; w[j] = tw;
#pragma unroll
                for (int k = 0; k < M; ++k) { double t = A[k * N + i]; A[k * N + i] = A[k * N + j]; A[k * N + j] = t; }
#pragma unroll
                for (int k = 0; k < N; ++k) { double t = V[k * N + i]; V[k * N + i] = V[k * N + j]; V[k * N + j] = t; }
            }
        }
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {
        if (w[i] > 0) {
            double inv = 1.0 / w[i];
#pragma unroll
            for (int k = 0; k < M; ++k) A[k * N + i] *= inv;
        }
    }
}

VO_DEV void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// svd_jacobi<M, N> executed by one whole wave with A [M*N], w [N], V [N*N] in LDS
// (row-major), M, N <= 64.  Same cyclic pair order and the same floating-point
// operations: every lane forms the three column sums in the scalar order from
// broadcast LDS reads (so all lanes take identical decisions), and lane k applies the
// rotation to row k of A and V.  Bit-identical to the scalar routine.
template <int M, int N>
VO_DEV void svd_jacobi_wave(double* A, double* w, double* V)
{
    const int lane = lane_id();
    for (int q = lane; q < N * N; q += 64) V[q] = (q / N == q % N) ? 1.0 : 0.0;
    wave_lds_sync();
    for (int sweep = 0; sweep < 60; ++sweep) {
        int changed = 0;
        for (int i = 0; i < N - 1; ++i) {
            for (int j = i + 1; j < N; ++j) {
                double alpha = 0, beta = 0, gamma = 0;
#pragma unroll
                for (int k = 0; k < M; ++k) {
                    double ai = A[k * N + i], aj = A[k * N + j];
                    alpha += ai * ai;
                    beta += aj * aj;
                    gamma += ai * aj;
                }
                if (alpha == 0.0 || beta == 0.0) continue;
                if (fabs(gamma) <= DBL_EPSILON * sqrt(alpha * beta)) continue;
                changed = 1;
                double zeta = (beta - alpha) / (2.0 * gamma);
                double t = 1.0 / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                if (zeta < 0) t = -t;
                double c = 1.0 / sqrt(1.0 + t * t);
                double s = c * t;
                if (lane < M) {
                    double ai = A[lane * N + i], aj = A[lane * N + j];
                    A[lane * N + i] = c * ai - s * aj;
                    A[lane * N + j] = s * ai + c * aj;
                }
                if (lane < N) {
                    double vi = V[lane * N + i], vj = V[lane * N + j];
                    V[lane * N + i] = c * vi - s * vj;
                    V[lane * N + j] = s * vi + c * vj;
                }
                wave_lds_sync();
            }
        }
        if (!changed) break;
    }
    for (int i = 0; i < N; ++i) {
        double s = 0;
#pragma unroll
        for (int k = 0; k < M; ++k) s += A[k * N + i] * A[k * N + i];
        if (lane == 0) w[i] = sqrt(s);
    }
    wave_lds_sync();
    for (int i = 0; i < N - 1; ++i) {
        int b = i;
        for (int j = i + 1; j < N; ++j) if (w[j] > w[b]) b = j;
        if (b != i) {
            wave_lds_sync();
            if (lane == 0) { double tw = w[i]; w[i] = w[b]; w[b] = tw; }
            if (lane < M) { double t = A[lane * N + i]; A[lane * N + i] = A[lane * N + b]; A[lane * N + b] = t; }
            if (lane < N) { double t = V[lane * N + i]; V[lane * N + i] = V[lane * N + b]; V[lane * N + b] = t; }
            wave_lds_sync();
        }
    }
    for (int i = 0; i < N; ++i) {
        if (w[i] > 0) {
            double inv = 1.0 / w[i];
            if (lane < M) A[lane * N + i] *= inv;
        }
    }
    wave_lds_sync();
}

// f64 lane exchange inside groups of four lanes (DPP quad_perm): xor 1 / xor 2
template <int CTRL>
VO_DEV double dpp_quad_f64(double v)
{
    const int2 w = __builtin_bit_cast(int2, v);
    int2 r;
    r.x = __builtin_amdgcn_update_dpp(0, w.x, CTRL, 0xf, 0xf, false);
    r.y = __builtin_amdgcn_update_dpp(0, w.y, CTRL, 0xf, 0xf, false);
    return __builtin_bit_cast(double, r);
}
VO_DEV double quad_sum_f64(double p)       // (p0 + p1) + (p2 + p3) in every lane of the quad
{
    const double s1 = p + dpp_quad_f64<0xB1>(p);      // quad_perm [1,0,3,2]
    return s1 + dpp_quad_f64<0x4E>(s1);               // quad_perm [2,3,0,1]
}

// Round-robin Jacobi SVD (oracle/vo_oracle_geom.c svd_jacobi_rr) by one wave, A [M*N], w [N],
// V [N*N] in LDS, N even, M a multiple of 4, 4 N <= 64.  Round r pairs the columns by the
// circle method; the N/2 pairs of a round are disjoint.  Lane 4 c + q (c < N) keeps rows
// q M/4 .. (q+1) M/4 - 1 of column c of A and of V in registers for all sweeps: per round it
// fetches its partner column's quarter with lane permutes, forms its partial sums serially,
// and the quad combines them as (p0 + p1) + (p2 + p3) -- the oracle's QUARTER_SUM; both
// columns of a pair form the same sums, the same rotation, and each quarter its own rotated
// rows: the oracle's operations on the same values, so bit-identical, with no LDS traffic or
// barrier inside the sweeps.  (cs is unused; kept for the callers' LDS layout.)
template <int M, int N>
VO_DEV void svd_jacobi_wave_rr(double* A, double* w, double* V, double* cs)
{
    static_assert(N % 2 == 0 && 4 * N <= 64 && M % 4 == 0 && N % 4 == 0, "round-robin SVD shape");
    (void)cs;
    constexpr int NP = N / 2, MQ = M / 4, NQ = N / 4;
    const int lane = lane_id();
    const bool act = lane < 4 * N;
    const int col = act ? lane >> 2 : 0, q = lane & 3;
    // partner of this lane's column in every round
    int prt[N - 1];
#pragma unroll
    for (int r = 0; r < N - 1; ++r) {
        prt[r] = col;
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            const int a = k == 0 ? 0 : ((k - 1 + r) % (N - 1)) + 1;
            const int b = ((N - 2 - k + r) % (N - 1)) + 1;
            if (a == col) prt[r] = b;
            if (b == col) prt[r] = a;
        }
    }
    double x[MQ], v[NQ];
#pragma unroll
    for (int k = 0; k < MQ; ++k) x[k] = A[(q * MQ + k) * N + col];
#pragma unroll
    for (int k = 0; k < NQ; ++k) v[k] = q * NQ + k == col ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 60; ++sweep) {
        bool changed = false;
#pragma unroll
        for (int r = 0; r < N - 1; ++r) {
            const int p = prt[r];
            const bool lo = col < p;           // this lane holds column i (= min of the pair)
            const int src = 4 * p + q;
            double px[MQ], pv[NQ];
#pragma unroll
            for (int k = 0; k < MQ; ++k) px[k] = __shfl(x[k], src, 64);
#pragma unroll
            for (int k = 0; k < NQ; ++k) pv[k] = __shfl(v[k], src, 64);
            double pa = 0, pb = 0, pg = 0;
#pragma unroll
            for (int k = 0; k < MQ; ++k) {
                const double ai = lo ? x[k] : px[k], aj = lo ? px[k] : x[k];
                pa += ai * ai;
                pb += aj * aj;
                pg += ai * aj;
            }
            const double alpha = quad_sum_f64(pa), beta = quad_sum_f64(pb), gamma = quad_sum_f64(pg);
            // skip test and rotation side by side, the rotation kept by selects (no branch:
            // the test's sqrt overlaps the rotation's division chain)
            const bool rot = alpha != 0.0 && beta != 0.0 && !(fabs(gamma) <= DBL_EPSILON * sqrt(alpha * beta));
            changed |= rot;
            {
                const double zeta = (beta - alpha) / (2.0 * gamma);
                const double u = fabs(zeta) + sqrt(1.0 + zeta * zeta);
                const double wn = sqrt(u * u + 1.0);
                const double c = u / wn;
                const double s = (zeta < 0 ? -1.0 : 1.0) / wn;
#pragma unroll
                for (int k = 0; k < MQ; ++k) {
                    const double xi = lo ? x[k] : px[k], xj = lo ? px[k] : x[k];
                    const double xr = lo ? c * xi - s * xj : s * xi + c * xj;
                    x[k] = rot ? xr : x[k];
                }
#pragma unroll
                for (int k = 0; k < NQ; ++k) {
                    const double vi = lo ? v[k] : pv[k], vj = lo ? pv[k] : v[k];
                    const double vr = lo ? c * vi - s * vj : s * vi + c * vj;
                    v[k] = rot ? vr : v[k];
                }
            }
        }
        if (__ballot(act && changed) == 0) break;
    }
    // column norms in the same quarter order, then the oracle's sort and normalisation
    double pn = 0;
#pragma unroll
    for (int k = 0; k < MQ; ++k) pn += x[k] * x[k];
    const double nn = quad_sum_f64(pn);
    if (act) {
#pragma unroll
        for (int k = 0; k < MQ; ++k) A[(q * MQ + k) * N + col] = x[k];
#pragma unroll
        for (int k = 0; k < NQ; ++k) V[(q * NQ + k) * N + col] = v[k];
        if (q == 0) w[col] = sqrt(nn);
    }
    wave_lds_sync();
    for (int i = 0; i < N - 1; ++i) {
        int b = i;
        for (int j = i + 1; j < N; ++j) if (w[j] > w[b]) b = j;
        if (b != i) {
            wave_lds_sync();
            if (lane == 0) { double tw = w[i]; w[i] = w[b]; w[b] = tw; }
            if (lane < M) { double t = A[lane * N + i]; A[lane * N + i] = A[lane * N + b]; A[lane * N + b] = t; }
            if (lane < N) { double t = V[lane * N + i]; V[lane * N + i] = V[lane * N + b]; V[lane * N + b] = t; }
            wave_lds_sync();
        }
    }
    for (int i = 0; i < N; ++i) {
        if (w[i] > 0) {
            double inv = 1.0 / w[i];
            if (lane < M) A[lane * N + i] *= inv;
        }
    }
    wave_lds_sync();
}

template <int M, int N>
VO_DEV void lsq_svd(const double* A_in, const double* b, double* x)
{
    double A[M * N], w[N], V[N * N];
#pragma unroll
    for (int i = 0; i < M * N; ++i) A[i] = A_in[i];
    svd_jacobi<M, N>(A, w, V);
    double thr = (w[0] > 0 ? w[0] : 0) * DBL_EPSILON * (M > N ? M : N);
    double utb[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        double s = 0;
#pragma unroll
        for (int k = 0; k < M; ++k) s += A[k * N + i] * b[k];
        utb[i] = (w[i] > thr) ? s / w[i] : 0.0;
    }
#pragma unroll
    for (int j = 0; j < N; ++j) {
        double s = 0;
#pragma unroll
        for (int i = 0; i < N; ++i) s += V[j * N + i] * utb[i];
        x[j] = s;
    }
}

VO_DEV double det3(const double* M)
{
    return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) +
           M[2] * (M[3] * M[7] - M[4] * M[6]);
}

VO_DEV void matmul3(const double* A, const double* B, double* C)
{
    double T[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            T[i * 3 + j] = A[i * 3 + 0] * B[0 * 3 + j] + A[i * 3 + 1] * B[1 * 3 + j] + A[i * 3 + 2] * B[2 * 3 + j];
    for (int i = 0; i < 9; ++i) C[i] = T[i];
}

// DLT null vector (cvTriangulatePoints): A = [x P3 - P1; y P3 - P2] of both views
VO_DEV void tri_one(const double* P1, const double* P2, double x1, double y1, double x2, double y2, double* X4)
{
    double A[16], w[4], V[16];
    for (int k = 0; k < 4; ++k) {
        A[0 * 4 + k] = x1 * P1[8 + k] - P1[k];
        A[1 * 4 + k] = y1 * P1[8 + k] - P1[4 + k];
        A[2 * 4 + k] = x2 * P2[8 + k] - P2[k];
        A[3 * 4 + k] = y2 * P2[8 + k] - P2[4 + k];
    }
    svd_jacobi<4, 4>(A, w, V);
    for (int k = 0; k < 4; ++k) X4[k] = V[k * 4 + 3];
}

VO_DEV void rodrigues_v2m(const double* r, double* R)
{
    double th = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    if (th < DBL_EPSILON) {
        for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0) ? 1.0 : 0.0;
        return;
    }
    double c = vcr_cos(th), s = vcr_sin(th), c1 = 1.0 - c, it = th ? 1.0 / th : 0.0;
    double x = r[0] * it, y = r[1] * it, z = r[2] * it;
    double rrt[9] = {x * x, x * y, x * z, x * y, y * y, y * z, x * z, y * z, z * z};
    double rx[9] = {0, -z, y, z, 0, -x, -y, x, 0};
    for (int i = 0; i < 9; ++i) R[i] = c * ((i % 4 == 0) ? 1.0 : 0.0) + c1 * rrt[i] + s * rx[i];
}

VO_DEV void rodrigues_m2v(const double* Rin, double* rv)
{
    double A[9], w[3], V[9], R[9];
    for (int i = 0; i < 9; ++i) A[i] = Rin[i];
    svd_jacobi<3, 3>(A, w, V);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            R[i * 3 + j] = A[i * 3 + 0] * V[j * 3 + 0] + A[i * 3 + 1] * V[j * 3 + 1] + A[i * 3 + 2] * V[j * 3 + 2];
    double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
    double s = sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    double c = (R[0] + R[4] + R[8] - 1) * 0.5;
    c = c > 1. ? 1. : c < -1. ? -1. : c;
    double th = vcr_acos(c);
    if (s < 1e-5) {
        if (c > 0) { rx = ry = rz = 0; }
        else {
            double t;
            t = (R[0] + 1) * 0.5; rx = sqrt(t > 0 ? t : 0.);
            t = (R[4] + 1) * 0.5; ry = sqrt(t > 0 ? t : 0.) * (R[1] < 0 ? -1. : 1.);
            t = (R[8] + 1) * 0.5; rz = sqrt(t > 0 ? t : 0.) * (R[2] < 0 ? -1. : 1.);
            if (fabs(rx) < fabs(ry) && fabs(rx) < fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
            th /= sqrt(rx * rx + ry * ry + rz * rz);
            rx *= th; ry *= th; rz *= th;
        }
    } else {
        double vth = 1 / (2 * s);
        vth *= th;
        rx *= vth; ry *= vth; rz *= vth;
    }
    rv[0] = rx; rv[1] = ry; rv[2] = rz;
}

// ------------------------------------------------------------------ real roots
VO_DEV double peval(const double* c, int deg, double x)
{
    double v = c[deg];
    for (int i = deg - 1; i >= 0; --i) v = v * x + c[i];
    return v;
}

VO_DEV double bracket_root(const double* c, const double* dc, int deg, double lo, double hi, double flo)
{
    double x = 0.5 * (lo + hi);
    for (int it = 0; it < 100; ++it) {
        double f = peval(c, deg, x);
        if (f == 0.0) return x;
        if ((f < 0) == (flo < 0)) lo = x; else hi = x;
        double d = peval(dc, deg - 1, x);
        double xn = (d != 0.0) ? x - f / d : 0.5 * (lo + hi);
        if (!(xn > lo && xn < hi)) xn = 0.5 * (lo + hi);
        if (xn == x || hi - lo <= 4.0 * DBL_EPSILON * fabs(x)) return xn;
        x = xn;
    }
    return x;
}

template <int D>
VO_DEV int real_roots(const double* c_in, int deg, double* roots);

template <>
VO_DEV int real_roots<2>(const double* c_in, int deg, double* roots)
{
    while (deg > 0 && c_in[deg] == 0.0) --deg;
    if (deg <= 0) return 0;
    double c[3];
    for (int i = 0; i <= deg; ++i) c[i] = c_in[i] / c_in[deg];
    if (deg == 1) { roots[0] = -c[0]; return 1; }
    double disc = c[1] * c[1] - 4.0 * c[0];
    if (disc < 0) return 0;
    double sq = sqrt(disc);
    double q = (c[1] >= 0) ? -0.5 * (c[1] + sq) : -0.5 * (c[1] - sq);
    double r0 = q, r1 = (q != 0.0) ? c[0] / q : 0.0;
    if (r0 > r1) { double t = r0; r0 = r1; r1 = t; }
    roots[0] = r0; roots[1] = r1;
    return 2;
}

template <int D>
VO_DEV int real_roots(const double* c_in, int deg, double* roots)
{
    while (deg > 0 && c_in[deg] == 0.0) --deg;
    if (deg <= 0) return 0;
    if (deg < D) return real_roots<D - 1>(c_in, deg, roots);
    double c[D + 1];
    for (int i = 0; i <= D; ++i) c[i] = c_in[i] / c_in[D];
    double dc[D];
    for (int i = 1; i <= D; ++i) dc[i - 1] = c[i] * i;
    double crit[D];
    int nc = real_roots<D - 1>(dc, D - 1, crit);
    double bound = 0;
    for (int i = 0; i < D; ++i) if (fabs(c[i]) > bound) bound = fabs(c[i]);
    bound += 1.0;
    double pts[D + 2];
    int np = 0;
    pts[np++] = -bound;
    for (int i = 0; i < nc; ++i) if (crit[i] > -bound && crit[i] < bound) pts[np++] = crit[i];
    pts[np++] = bound;
    int nr = 0;
    double fprev = peval(c, D, pts[0]);
    for (int k = 1; k < np; ++k) {
        double f = peval(c, D, pts[k]);
        if (f == 0.0) { roots[nr++] = pts[k]; }
        else if (fprev != 0.0 && ((f < 0) != (fprev < 0))) roots[nr++] = bracket_root(c, dc, D, pts[k - 1], pts[k], fprev);
        fprev = f;
    }
    return nr;
}

// real_roots<D> computed by the four lanes of a quad together (sub = lane & 3; every lane of
// the quad calls it with the same coefficients): lane k brackets interval k + 1 of the serial
// walk -- the same peval / bracket_root calls on the same values -- and the roots are gathered
// in interval order, so the result is bit-identical to real_roots<D> while the quad's serial
// chain is one bracket per degree instead of up to D.
template <int D>
VO_DEV int real_roots_q(const double* c_in, int deg, double* roots, int sub);

template <>
VO_DEV int real_roots_q<2>(const double* c_in, int deg, double* roots, int sub)
{
    (void)sub;
    return real_roots<2>(c_in, deg, roots);
}

template <int D>
VO_DEV int real_roots_q(const double* c_in, int deg, double* roots, int sub)
{
    while (deg > 0 && c_in[deg] == 0.0) --deg;
    if (deg <= 0) return 0;
    if (deg < D) return real_roots_q<D - 1>(c_in, deg, roots, sub);
    double c[D + 1];
    for (int i = 0; i <= D; ++i) c[i] = c_in[i] / c_in[D];
    double dc[D];
    for (int i = 1; i <= D; ++i) dc[i - 1] = c[i] * i;
    double crit[D];
    int nc = real_roots_q<D - 1>(dc, D - 1, crit, sub);
    double bound = 0;
    for (int i = 0; i < D; ++i) if (fabs(c[i]) > bound) bound = fabs(c[i]);
    bound += 1.0;
    double pts[D + 2];
    int np = 0;
    pts[np++] = -bound;
    for (int i = 0; i < nc; ++i) if (crit[i] > -bound && crit[i] < bound) pts[np++] = crit[i];
    pts[np++] = bound;
    // interval k = sub + 1 of the serial walk (fprev there is peval(pts[k - 1]))
    double rk = 0.0;
    int has = 0;
    {
        const int k = sub + 1;
        if (k < np) {
            double lo = pts[0], hi = pts[1];
#pragma unroll
            for (int i = 1; i < D + 1; ++i)
                if (i == k) { lo = pts[i - 1]; hi = pts[i]; }         // constant indices
            const double fprev = peval(c, D, lo);
            const double f = peval(c, D, hi);
            if (f == 0.0) { rk = hi; has = 1; }
            else if (fprev != 0.0 && ((f < 0) != (fprev < 0))) { rk = bracket_root(c, dc, D, lo, hi, fprev); has = 1; }
        }
    }
    const int base = lane_id() & ~3;
    int nr = 0;
#pragma unroll
    for (int j = 0; j < D; ++j) {
        const int hj = __shfl(has, base | j, 64);
        const double rj = __shfl(rk, base | j, 64);
        if (j + 1 < np && hj) roots[nr++] = rj;
    }
    return nr;
}

// ------------------------------------------------------------------ P3P
struct CamK {
    double fx, fy, cx, cy, ifx, ify, cx_fx, cy_fx;
};

VO_DEV CamK camk(const double* K)
{
    CamK k;
    k.fx = K[0]; k.fy = K[4]; k.cx = K[2]; k.cy = K[5];
    k.ifx = 1.0 / k.fx; k.ify = 1.0 / k.fy;
    k.cx_fx = k.cx / k.fx; k.cy_fx = k.cy / k.fy;
    return k;
}

VO_DEV void jacobi_eig4(double* S, double* ev, double* U)
{
#pragma unroll
    for (int i = 0; i < 16; ++i) U[i] = (i % 5 == 0) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 50; ++sweep) {
        double off = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = i + 1; j < 4; ++j) off += S[i * 4 + j] * S[i * 4 + j];
        if (off < 1e-300) break;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
#pragma unroll
            for (int q = p + 1; q < 4; ++q) {
                double apq = S[p * 4 + q];
                if (apq == 0.0) continue;
                double theta = (S[q * 4 + q] - S[p * 4 + p]) / (2.0 * apq);
                double t = 1.0 / (fabs(theta) + sqrt(theta * theta + 1.0));
                if (theta < 0) t = -t;
                double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    double skp = S[k * 4 + p], skq = S[k * 4 + q];
                    S[k * 4 + p] = c * skp - s * skq;
                    S[k * 4 + q] = s * skp + c * skq;
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    double spk = S[p * 4 + k], sqk = S[q * 4 + k];
                    S[p * 4 + k] = c * spk - s * sqk;
                    S[q * 4 + k] = s * spk + c * sqk;
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    double ukp = U[k * 4 + p], ukq = U[k * 4 + q];
                    U[k * 4 + p] = c * ukp - s * ukq;
                    U[k * 4 + q] = s * ukp + c * ukq;
                }
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) ev[i] = S[i * 4 + i];
}

VO_DEV void align_horn(const double M[3][3], const double P[3][3], double* R, double* T)
{
    double cm[3], cp[3], s[9];
    for (int j = 0; j < 3; ++j) {
        cm[j] = (M[0][j] + M[1][j] + M[2][j]) / 3;
        cp[j] = (P[0][j] + P[1][j] + P[2][j]) / 3;
    }
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b)
            s[a * 3 + b] = (P[0][a] * M[0][b] + P[1][a] * M[1][b] + P[2][a] * M[2][b]) / 3 - cm[b] * cp[a];
    double N[16], ev[4], U[16];
    N[0] = s[0] + s[4] + s[8];
    N[5] = s[0] - s[4] - s[8];
    N[10] = s[4] - s[8] - s[0];
    N[15] = s[8] - s[0] - s[4];
    N[1] = N[4] = s[5] - s[7];
    N[2] = N[8] = s[6] - s[2];
    N[3] = N[12] = s[1] - s[3];
    N[6] = N[9] = s[3] + s[1];
    N[7] = N[13] = s[6] + s[2];
    N[11] = N[14] = s[7] + s[5];
    jacobi_eig4(N, ev, U);
    // column of the largest eigenvalue (first on ties), selected with constant indices
    double q0 = U[0], q1 = U[4], q2 = U[8], q3 = U[12], eb = ev[0];
#pragma unroll
    for (int i = 1; i < 4; ++i)
        if (ev[i] > eb) { eb = ev[i]; q0 = U[i]; q1 = U[4 + i]; q2 = U[8 + i]; q3 = U[12 + i]; }
    R[0] = q0 * q0 + q1 * q1 - q2 * q2 - q3 * q3;
    R[1] = 2. * (q1 * q2 - q0 * q3);
    R[2] = 2. * (q1 * q3 + q0 * q2);
    R[3] = 2. * (q1 * q2 + q0 * q3);
    R[4] = q0 * q0 + q2 * q2 - q1 * q1 - q3 * q3;
    R[5] = 2. * (q2 * q3 - q0 * q1);
    R[6] = 2. * (q1 * q3 - q0 * q2);
    R[7] = 2. * (q2 * q3 + q0 * q1);
    R[8] = q0 * q0 + q3 * q3 - q1 * q1 - q2 * q2;
    for (int i = 0; i < 3; ++i) T[i] = cm[i] - (R[i * 3] * cp[0] + R[i * 3 + 1] * cp[1] + R[i * 3 + 2] * cp[2]);
}

// sub < 0: serial root finder; sub = lane & 3: the quad-cooperative one (identical roots)
VO_DEV int p3p_lengths(double L[4][3], const double d[3], const double cs[3], int sub = -1)
{
    double p = cs[0] * 2, q = cs[1] * 2, r = cs[2] * 2;
    double inv_d22 = 1. / (d[2] * d[2]);
    double a = inv_d22 * (d[0] * d[0]);
    double b = inv_d22 * (d[1] * d[1]);
    if (p * p + q * q + r * r - p * q * r - 1 == 0) return 0;
    double n2 = 1 - a - b, n1 = (a - 1) * q, n0 = 1 - a + b;
    double A = n2 * n2 - a * b * r * r;
    if (A == 0) return 0;
    double Nn[3] = {n0, n1, n2};
    double NN[5] = {0, 0, 0, 0, 0};
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) NN[i + j] += Nn[i] * Nn[j];
    double xLp[3] = {0, p, -r};
    double LL[3] = {p * p, -2 * p * r, r * r};
    double Qq[3] = {1, -q, 1 - b};
    double c[5];
    for (int i = 0; i < 5; ++i) c[i] = NN[i];
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) if (i + j < 5) c[i + j] -= b * r * Nn[i] * xLp[j];
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) c[i + j] -= b * Qq[i] * LL[j];
    double xs[4];
    int nr = sub < 0 ? real_roots<4>(c, 4, xs) : real_roots_q<4>(c, 4, xs, sub);
    int ns = 0;
    for (int i = 0; i < nr; ++i) {
        double x = xs[i];
        if (x <= 0) continue;
        double den = b * (p - r * x);
        if (den == 0) continue;
        double y = (n2 * x * x + n1 * x + n0) / den;
        if (y <= 0) continue;
        double v = x * x + y * y - x * y * r;
        if (v <= 0) continue;
        double Z = d[2] / sqrt(v);
        L[ns][0] = x * Z;
        L[ns][1] = y * Z;
        L[ns][2] = Z;
        ++ns;
    }
    return ns;
}

VO_DEV void p3p_reproject_input(const CamK& k, double u, double v, double* uo, double* vo)
{
    float un = (float)((u - k.cx) * k.ifx);
    float vn = (float)((v - k.cy) * k.ify);
    *uo = (double)un * k.fx + k.cx;
    *vo = (double)vn * k.fy + k.cy;
}

// Solution `sol` of a 4-point P3P, for the lane-per-solution layout of k_pnp_ransac: the
// same bearing/length computation as p3p_solve4 (every lane of a hypothesis runs it on the
// same data), then one align_horn.  Returns 0 when the quartic gave fewer solutions;
// otherwise R, T and the 4th-point error e that p3p_solve4 ranks the solutions by.
VO_DEV int p3p_solution(const CamK& k, const double* obj, const double* img_px, int sol, double* R, double* T,
                        double* e)
{
    double mu[4], mv[4], mk[3];
    for (int i = 0; i < 4; ++i) {
        double u, v;
        p3p_reproject_input(k, img_px[2 * i], img_px[2 * i + 1], &u, &v);
        mu[i] = k.ifx * u - k.cx_fx;
        mv[i] = k.ify * v - k.cy_fx;
    }
    for (int i = 0; i < 3; ++i) {
        double nrm = sqrt(mu[i] * mu[i] + mv[i] * mv[i] + 1);
        mk[i] = 1. / nrm;
        mu[i] *= mk[i];
        mv[i] *= mk[i];
    }
    const double* X = obj;
    double dist[3], cs[3];
    dist[0] = sqrt((X[3] - X[6]) * (X[3] - X[6]) + (X[4] - X[7]) * (X[4] - X[7]) + (X[5] - X[8]) * (X[5] - X[8]));
    dist[1] = sqrt((X[0] - X[6]) * (X[0] - X[6]) + (X[1] - X[7]) * (X[1] - X[7]) + (X[2] - X[8]) * (X[2] - X[8]));
    dist[2] = sqrt((X[0] - X[3]) * (X[0] - X[3]) + (X[1] - X[4]) * (X[1] - X[4]) + (X[2] - X[5]) * (X[2] - X[5]));
    cs[0] = mu[1] * mu[2] + mv[1] * mv[2] + mk[1] * mk[2];
    cs[1] = mu[0] * mu[2] + mv[0] * mv[2] + mk[0] * mk[2];
    cs[2] = mu[0] * mu[1] + mv[0] * mv[1] + mk[0] * mk[1];
    double L[4][3];
    const int n = p3p_lengths(L, dist, cs, sol);      // the quad's four lanes find the roots together
    if (sol >= n) return 0;
    double l0 = 0, l1 = 0, l2 = 0;          // L[sol] selected with constant indices
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (i == sol) { l0 = L[i][0]; l1 = L[i][1]; l2 = L[i][2]; }
    const double ls[3] = {l0, l1, l2};
    double M[3][3], P[3][3];
    for (int j = 0; j < 3; ++j) {
        M[j][0] = ls[j] * mu[j];
        M[j][1] = ls[j] * mv[j];
        M[j][2] = ls[j] * mk[j];
        P[j][0] = X[3 * j]; P[j][1] = X[3 * j + 1]; P[j][2] = X[3 * j + 2];
    }
    align_horn(M, P, R, T);
    double X3 = R[0] * X[9] + R[1] * X[10] + R[2] * X[11] + T[0];
    double Y3 = R[3] * X[9] + R[4] * X[10] + R[5] * X[11] + T[1];
    double Z3 = R[6] * X[9] + R[7] * X[10] + R[8] * X[11] + T[2];
    *e = (X3 / Z3 - mu[3]) * (X3 / Z3 - mu[3]) + (Y3 / Z3 - mv[3]) * (Y3 / Z3 - mv[3]);
    return 1;
}

// 4-point P3P (solvePnP SOLVEPNP_P3P): obj 4x3, img_px 4x2 (doubles from float inputs)
VO_DEV int p3p_solve4(const CamK& k, const double* obj, const double* img_px, double* Rb, double* tb)
{
    double mu[4], mv[4], mk[3];
    for (int i = 0; i < 4; ++i) {
        double u, v;
        p3p_reproject_input(k, img_px[2 * i], img_px[2 * i + 1], &u, &v);
        mu[i] = k.ifx * u - k.cx_fx;
        mv[i] = k.ify * v - k.cy_fx;
    }
    for (int i = 0; i < 3; ++i) {
        double nrm = sqrt(mu[i] * mu[i] + mv[i] * mv[i] + 1);
        mk[i] = 1. / nrm;
        mu[i] *= mk[i];
        mv[i] *= mk[i];
    }
    const double* X = obj;
    double dist[3], cs[3];
    dist[0] = sqrt((X[3] - X[6]) * (X[3] - X[6]) + (X[4] - X[7]) * (X[4] - X[7]) + (X[5] - X[8]) * (X[5] - X[8]));
    dist[1] = sqrt((X[0] - X[6]) * (X[0] - X[6]) + (X[1] - X[7]) * (X[1] - X[7]) + (X[2] - X[8]) * (X[2] - X[8]));
    dist[2] = sqrt((X[0] - X[3]) * (X[0] - X[3]) + (X[1] - X[4]) * (X[1] - X[4]) + (X[2] - X[5]) * (X[2] - X[5]));
    cs[0] = mu[1] * mu[2] + mv[1] * mv[2] + mk[1] * mk[2];
    cs[1] = mu[0] * mu[2] + mv[0] * mv[2] + mk[0] * mk[2];
    cs[2] = mu[0] * mu[1] + mv[0] * mv[1] + mk[0] * mk[1];
    double L[4][3];
    int n = p3p_lengths(L, dist, cs);
    int best = -1;
    double best_err = 0;
    for (int i = 0; i < n; ++i) {
        double M[3][3], P[3][3], R[9], T[3];
        for (int j = 0; j < 3; ++j) {
            M[j][0] = L[i][j] * mu[j];
            M[j][1] = L[i][j] * mv[j];
            M[j][2] = L[i][j] * mk[j];
            P[j][0] = X[3 * j]; P[j][1] = X[3 * j + 1]; P[j][2] = X[3 * j + 2];
        }
        align_horn(M, P, R, T);
        double X3 = R[0] * X[9] + R[1] * X[10] + R[2] * X[11] + T[0];
        double Y3 = R[3] * X[9] + R[4] * X[10] + R[5] * X[11] + T[1];
        double Z3 = R[6] * X[9] + R[7] * X[10] + R[8] * X[11] + T[2];
        double e = (X3 / Z3 - mu[3]) * (X3 / Z3 - mu[3]) + (Y3 / Z3 - mv[3]) * (Y3 / Z3 - mv[3]);
        if (best < 0 || e < best_err) {
            best = i;
            best_err = e;
            for (int q = 0; q < 9; ++q) Rb[q] = R[q];
            for (int q = 0; q < 3; ++q) tb[q] = T[q];
        }
    }
    return best >= 0;
}

// projectPoints (zero distortion) -> float, squared pixel error in float
VO_DEV float pnp_err(const double* R, const double* t, const CamK& k, float X0, float X1, float X2, float u, float v)
{
    double Xd = X0, Yd = X1, Zd = X2;
    double xx = R[0] * Xd + R[1] * Yd + R[2] * Zd + t[0];
    double yy = R[3] * Xd + R[4] * Yd + R[5] * Zd + t[1];
    double zz = R[6] * Xd + R[7] * Yd + R[8] * Zd + t[2];
    zz = zz != 0.0 ? 1. / zz : 1;
    xx *= zz;
    yy *= zz;
    float pu = (float)(xx * k.fx + k.cx);
    float pv = (float)(yy * k.fy + k.cy);
    float du = u - pu, dv = v - pv;
    return du * du + dv * dv;
}

// RANSACUpdateNumIters split in two: the numerator log(max(1 - p, DBL_MIN)) depends only on the
// confidence, so a RANSAC loop forms it once and passes it to every update (same values as
// forming it per call; the early `denom < DBL_MIN` return does not depend on it)
VO_DEV double ransac_log_num(double p)
{
    p = p < 0 ? 0 : (p > 1 ? 1 : p);
    return vcr_log(1. - p > DBL_MIN ? 1. - p : DBL_MIN);
}
// ... and the denominator part, which depends only on the inlier ratio: 0 when
// 1 - (1 - ep)^mp < DBL_MIN (the update then returns 0), else 1 with *ld = log(1 - (1 - ep)^mp).
// A RANSAC loop can form it for a batch of hypotheses in parallel and apply the sequential
// rule with ransac_niters_fin afterwards (the same operations on the same values).
VO_DEV int ransac_niters_den(double ep, int model_points, double* ld)
{
    ep = ep < 0 ? 0 : (ep > 1 ? 1 : ep);
    const double denom = 1. - vcr_powi(1. - ep, model_points);
    if (denom < DBL_MIN) return 0;
    *ld = vcr_log(denom);
    return 1;
}
VO_DEV int ransac_niters_fin(double lnum, int ok, double ld, int max_iters)
{
    if (!ok) return 0;
    return (ld >= 0 || -lnum >= max_iters * (-ld)) ? max_iters : (int)rint(lnum / ld);
}
VO_DEV int ransac_update_niters_ln(double lnum, double ep, int model_points, int max_iters)
{
    double ld = 0.0;
    const int ok = ransac_niters_den(ep, model_points, &ld);
    return ransac_niters_fin(lnum, ok, ld, max_iters);
}
VO_DEV int ransac_update_niters(double p, double ep, int model_points, int max_iters)
{
    return ransac_update_niters_ln(ransac_log_num(p), ep, model_points, max_iters);
}

VO_DEV float sampson_err(const double* E, double x1, double y1, double x2, double y2)
{
    double Ex1[3] = {E[0] * x1 + E[1] * y1 + E[2], E[3] * x1 + E[4] * y1 + E[5], E[6] * x1 + E[7] * y1 + E[8]};
    double Etx2[3] = {E[0] * x2 + E[3] * y2 + E[6], E[1] * x2 + E[4] * y2 + E[7], E[2] * x2 + E[5] * y2 + E[8]};
    double x2tEx1 = x2 * Ex1[0] + y2 * Ex1[1] + Ex1[2];
    double a = Ex1[0] * Ex1[0], b = Ex1[1] * Ex1[1], c = Etx2[0] * Etx2[0], d = Etx2[1] * Etx2[1];
    return (float)(x2tEx1 * x2tEx1 / (a + b + c + d));
}

}  // namespace vg
