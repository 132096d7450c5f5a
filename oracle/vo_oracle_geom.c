/*
 * vo_oracle_geom.c -- CPU ORACLE (test infrastructure only; see vo_oracle.h).
 *
 * Restates the OpenCV 4.6 geometry that the reference calls:
 *   VisualOdometryPipeLine.py:188  cv2.triangulatePoints          
 *   VisualOdometryPipeLine.py:308  cv2.findEssentialMat RANSAC    
 *   VisualOdometryPipeLine.py:315  cv2.recoverPose                
 *   VisualOdometryPipeLine.py:343  cv2.solvePnPRansac SOLVEPNP_P3P
 *   VisualOdometryPipeLine.py:354  cv2.Rodrigues                  
 *
 * Algorithms: one-sided Jacobi SVD (OpenCV uses JacobiSVD for these small sizes),
 * Gao's P3P quartic (derived here in its "E2" form, see tests), Horn's quaternion
 * absolute orientation, EPnP (Lepetit et al.) with 3 beta approximations + 5 Gauss-
 * Newton steps, Nister's 5-point solver via a 10x20 action-matrix elimination and
 * OpenCV's Weierstrass (solvePoly) root finder, RANSAC with cv::RNG((uint64)-1).
 *
 * Documented deviations (mirrored by the HIP path):
 *   - RANSAC-PnP scores hypotheses with the rotation matrix directly (OpenCV scores
 *     via rvec -> Rodrigues -> R, a ~1e-16 relative round trip).
 *   - Real quartic roots (P3P) come from a bracketed Newton/bisection solver that
 *     uses only + - * / sqrt (OpenCV: closed-form Ferrari).
 *   - Sums over points inside EPnP use a fixed order -- item i goes to partial
 *     (i % 64), then a pairwise tree 32,16,..,1 -- which is exactly one 64-lane
 *     wave's strided accumulation + shuffle tree on the GPU.
 */
#include "vo_oracle.h"
#include "../monocular_visual_odometry_va4mr_amd/csrc/vo_crmath.h"   /* correctly rounded cos/sin/acos/log/pow (shared with the kernels) */

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define NPART 64

/* ================================================================ linalg */

/* One-sided Jacobi SVD of A (m x n, row-major, m >= 1).  On return A holds U*diag(w)
 * columns normalised to U (columns sorted by w descending), w[n], V (n x n, columns). */
static void svd_jacobi(double* A, int m, int n, double* w, double* V)
{
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) V[i * n + j] = (i == j) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 60; ++sweep) {
        int changed = 0;
        for (int i = 0; i < n - 1; ++i) {
            for (int j = i + 1; j < n; ++j) {
                double alpha = 0, beta = 0, gamma = 0;
                for (int k = 0; k < m; ++k) {
                    double ai = A[k * n + i], aj = A[k * n + j];
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
                for (int k = 0; k < m; ++k) {
                    double ai = A[k * n + i], aj = A[k * n + j];
                    A[k * n + i] = c * ai - s * aj;
                    A[k * n + j] = s * ai + c * aj;
                }
                for (int k = 0; k < n; ++k) {
                    double vi = V[k * n + i], vj = V[k * n + j];
                    V[k * n + i] = c * vi - s * vj;
                    V[k * n + j] = s * vi + c * vj;
                }
            }
        }
        if (!changed) break;
    }
    for (int i = 0; i < n; ++i) {
        double s = 0;
        for (int k = 0; k < m; ++k) s += A[k * n + i] * A[k * n + i];
        w[i] = sqrt(s);
    }
    /* selection sort descending, swapping columns of A and V */
    for (int i = 0; i < n - 1; ++i) {
        int b = i;
        for (int j = i + 1; j < n; ++j) if (w[j] > w[b]) b = j;
        if (b != i) {
            double tw = w[i]; w[i] = w[b]; w[b] = tw;
            for (int k = 0; k < m; ++k) { double t = A[k * n + i]; A[k * n + i] = A[k * n + b]; A[k * n + b] = t; }
            for (int k = 0; k < n; ++k) { double t = V[k * n + i]; V[k * n + i] = V[k * n + b]; V[k * n + b] = t; }
        }
    }
    for (int i = 0; i < n; ++i) {
        if (w[i] > 0) {
            double inv = 1.0 / w[i];
            for (int k = 0; k < m; ++k) A[k * n + i] *= inv;
        }
    }
}

/* Sum over k of f(k) for k = 0..m-1 (m a multiple of 4) in the order the GPU's quad of lanes
 * forms it: four serial partial sums over the row quarters, then (p0 + p1) + (p2 + p3). */
#define QUARTER_SUM(res, m, expr)                                              \
    do {                                                                       \
        double qs_[4] = {0, 0, 0, 0};                                          \
        const int qm_ = (m) / 4;                                               \
        for (int q_ = 0; q_ < 4; ++q_)                                         \
            for (int k = q_ * qm_; k < (q_ + 1) * qm_; ++k) qs_[q_] += (expr); \
        (res) = (qs_[0] + qs_[1]) + (qs_[2] + qs_[3]);                         \
    } while (0)

/* Round-robin ("parallel ordering") one-sided Jacobi SVD for even n and m a multiple of 4
 * (EPnP's 12x12 M^T M).  Each sweep runs n-1 rounds; round r pairs the columns by the circle
 * method (column 0 fixed, the others rotated by r), so a round's rotations touch disjoint
 * column pairs and may be applied in any order (or all at once, as the GPU does).  The GPU
 * gives every column four lanes (one row quarter each), so the column dot products are
 * quarter-wise partial sums combined pairwise (QUARTER_SUM), and the rotation is formed as
 * u = |zeta| + sqrt(1 + zeta^2), w = sqrt(u^2 + 1), c = u / w, s = sign(zeta) / w -- the same
 * rotation as t = sign / u, c = 1 / sqrt(1 + t^2), s = c t, one dependent division shorter.
 * Stopping rule, sort and normalisation as svd_jacobi.  (OpenCV's JacobiSVD uses the cyclic
 * order and its own summation; the decompositions agree to rounding -- OpenCV-level parity is
 * unpinned anyway, and the GPU follows this order exactly.) */
/* The round-2 form of svd_jacobi_rr -- serial column sums k = 0..m-1 and the rotation as
 * t = sign / u, c = 1 / sqrt(1 + t^2), s = c t -- kept as an independent cross-check of the
 * round-3 form (QUARTER_SUM + u / wn) that the GPU follows and every golden assumes
 * (vo_o_set_svd_form(1); tests/test_oracle_kat.py, tools/svd_form_trajectory.py). */
static int g_svd_form = 0;
void vo_o_set_svd_form(int form) { g_svd_form = form; }
int vo_o_get_svd_form(void) { return g_svd_form; }

#define SERIAL_SUM(res, m, expr)                                               \
    do {                                                                       \
        double ss_ = 0;                                                        \
        for (int k = 0; k < (m); ++k) ss_ += (expr);                           \
        (res) = ss_;                                                           \
    } while (0)

static void svd_jacobi_rr(double* A, int m, int n, double* w, double* V)
{
    const int serial = g_svd_form == 1;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) V[i * n + j] = (i == j) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 60; ++sweep) {
        int changed = 0;
        for (int r = 0; r < n - 1; ++r) {
            for (int q = 0; q < n / 2; ++q) {
                const int a = q == 0 ? 0 : ((q - 1 + r) % (n - 1)) + 1;
                const int b = ((n - 2 - q + r) % (n - 1)) + 1;
                const int i = a < b ? a : b, j = a < b ? b : a;
                double alpha, beta, gamma;
                if (serial) {
                    SERIAL_SUM(alpha, m, A[k * n + i] * A[k * n + i]);
                    SERIAL_SUM(beta, m, A[k * n + j] * A[k * n + j]);
                    SERIAL_SUM(gamma, m, A[k * n + i] * A[k * n + j]);
                } else {
                    QUARTER_SUM(alpha, m, A[k * n + i] * A[k * n + i]);
                    QUARTER_SUM(beta, m, A[k * n + j] * A[k * n + j]);
                    QUARTER_SUM(gamma, m, A[k * n + i] * A[k * n + j]);
                }
                if (alpha == 0.0 || beta == 0.0) continue;
                if (fabs(gamma) <= DBL_EPSILON * sqrt(alpha * beta)) continue;
                changed = 1;
                const double zeta = (beta - alpha) / (2.0 * gamma);
                double c, s;
                if (serial) {
                    double t = 1.0 / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                    if (zeta < 0) t = -t;
                    c = 1.0 / sqrt(1.0 + t * t);
                    s = c * t;
                } else {
                    const double u = fabs(zeta) + sqrt(1.0 + zeta * zeta);
                    const double wn = sqrt(u * u + 1.0);
                    c = u / wn;
                    s = (zeta < 0 ? -1.0 : 1.0) / wn;
                }
                for (int k = 0; k < m; ++k) {
                    double ai = A[k * n + i], aj = A[k * n + j];
                    A[k * n + i] = c * ai - s * aj;
                    A[k * n + j] = s * ai + c * aj;
                }
                for (int k = 0; k < n; ++k) {
                    double vi = V[k * n + i], vj = V[k * n + j];
                    V[k * n + i] = c * vi - s * vj;
                    V[k * n + j] = s * vi + c * vj;
                }
            }
        }
        if (!changed) break;
    }
    for (int i = 0; i < n; ++i) {
        double s;
        if (serial) SERIAL_SUM(s, m, A[k * n + i] * A[k * n + i]);
        else QUARTER_SUM(s, m, A[k * n + i] * A[k * n + i]);
        w[i] = sqrt(s);
    }
    for (int i = 0; i < n - 1; ++i) {
        int b = i;
        for (int j = i + 1; j < n; ++j) if (w[j] > w[b]) b = j;
        if (b != i) {
            double tw = w[i]; w[i] = w[b]; w[b] = tw;
            for (int k = 0; k < m; ++k) { double t = A[k * n + i]; A[k * n + i] = A[k * n + b]; A[k * n + b] = t; }
            for (int k = 0; k < n; ++k) { double t = V[k * n + i]; V[k * n + i] = V[k * n + b]; V[k * n + b] = t; }
        }
    }
    for (int i = 0; i < n; ++i) {
        if (w[i] > 0) {
            double inv = 1.0 / w[i];
            for (int k = 0; k < m; ++k) A[k * n + i] *= inv;
        }
    }
}

/* least squares min ||A x - b|| via SVD pseudo-inverse (cv::solve DECOMP_SVD) */
static void lsq_svd(const double* A_in, int m, int n, const double* b, double* x)
{
    double A[64], w[8], V[64];
    memcpy(A, A_in, sizeof(double) * m * n);
    svd_jacobi(A, m, n, w, V);
    double thr = (w[0] > 0 ? w[0] : 0) * DBL_EPSILON * (m > n ? m : n);
    double utb[8];
    for (int i = 0; i < n; ++i) {
        double s = 0;
        for (int k = 0; k < m; ++k) s += A[k * n + i] * b[k];
        utb[i] = (w[i] > thr) ? s / w[i] : 0.0;
    }
    for (int j = 0; j < n; ++j) {
        double s = 0;
        for (int i = 0; i < n; ++i) s += V[j * n + i] * utb[i];
        x[j] = s;
    }
}

static double det3(const double* M)
{
    return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) +
           M[2] * (M[3] * M[7] - M[4] * M[6]);
}

static void matmul3(const double* A, const double* B, double* C)
{
    double T[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            T[i * 3 + j] = A[i * 3 + 0] * B[0 * 3 + j] + A[i * 3 + 1] * B[1 * 3 + j] + A[i * 3 + 2] * B[2 * 3 + j];
    memcpy(C, T, sizeof T);
}

/* Gaussian elimination with partial pivoting: solve A X = B, A n x n, B n x m (row-major). */
static int gauss_solve(double* A, int n, double* B, int m)
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

/* ================================================================ triangulation */

/* cvTriangulatePoints: A = [x P3 - P1; y P3 - P2] for both views, null vector of A. */
static void tri_one(const double* P1, const double* P2, double x1, double y1, double x2,
                    double y2, double* X4)
{
    double A[16], w[4], V[16];
    for (int k = 0; k < 4; ++k) {
        A[0 * 4 + k] = x1 * P1[8 + k] - P1[k];
        A[1 * 4 + k] = y1 * P1[8 + k] - P1[4 + k];
        A[2 * 4 + k] = x2 * P2[8 + k] - P2[k];
        A[3 * 4 + k] = y2 * P2[8 + k] - P2[4 + k];
    }
    svd_jacobi(A, 4, 4, w, V);
    for (int k = 0; k < 4; ++k) X4[k] = V[k * 4 + 3];
}

int vo_o_triangulate(const double* P1, const double* P2, const float* x1, const float* x2,
                     int n, float* out4n)
{
    if (!P1 || !P2 || (n > 0 && (!x1 || !x2 || !out4n))) return VO_O_EARG;
    for (int i = 0; i < n; ++i) {
        double X[4];
        tri_one(P1, P2, x1[2 * i], x1[2 * i + 1], x2[2 * i], x2[2 * i + 1], X);
        for (int k = 0; k < 4; ++k) out4n[k * n + i] = (float)X[k];
    }
    return VO_O_OK;
}

int vo_o_triangulate_d(const double* P1, const double* P2, const double* x1, const double* x2,
                       int n, double* out4n)
{
    for (int i = 0; i < n; ++i) {
        double X[4];
        tri_one(P1, P2, x1[2 * i], x1[2 * i + 1], x2[2 * i], x2[2 * i + 1], X);
        for (int k = 0; k < 4; ++k) out4n[k * n + i] = X[k];
    }
    return VO_O_OK;
}

/* ================================================================ Rodrigues */
int vo_o_rodrigues_v2m(const double* r, double* R)
{
    double th = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    if (th < DBL_EPSILON) {
        for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0) ? 1.0 : 0.0;
        return VO_O_OK;
    }
    double c = vcr_cos(th), s = vcr_sin(th), c1 = 1.0 - c, it = th ? 1.0 / th : 0.0;
    double x = r[0] * it, y = r[1] * it, z = r[2] * it;
    double rrt[9] = {x * x, x * y, x * z, x * y, y * y, y * z, x * z, y * z, z * z};
    double rx[9] = {0, -z, y, z, 0, -x, -y, x, 0};
    for (int i = 0; i < 9; ++i) R[i] = c * ((i % 4 == 0) ? 1.0 : 0.0) + c1 * rrt[i] + s * rx[i];
    return VO_O_OK;
}

int vo_o_rodrigues_m2v(const double* Rin, double* rv)
{
    double A[9], w[3], V[9], R[9];
    memcpy(A, Rin, sizeof A);
    svd_jacobi(A, 3, 3, w, V);
    /* R = U V^T (orthogonalise) */
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
    return VO_O_OK;
}

/* ================================================================ real poly roots */

static double peval(const double* c, int deg, double x)
{
    double v = c[deg];
    for (int i = deg - 1; i >= 0; --i) v = v * x + c[i];
    return v;
}

/* root of c in [lo, hi] with f(lo), f(hi) of opposite sign: safeguarded Newton */
static double bracket_root(const double* c, const double* dc, int deg, double lo, double hi,
                           double flo)
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

/* real roots of sum c[i] x^i (deg <= 4, c[deg] != 0), ascending; returns count */
static int real_roots(const double* c_in, int deg, double* roots)
{
    while (deg > 0 && c_in[deg] == 0.0) --deg;
    if (deg <= 0) return 0;
    double c[5];
    for (int i = 0; i <= deg; ++i) c[i] = c_in[i] / c_in[deg];
    if (deg == 1) { roots[0] = -c[0]; return 1; }
    if (deg == 2) {
        double disc = c[1] * c[1] - 4.0 * c[0];
        if (disc < 0) return 0;
        double sq = sqrt(disc);
        double q = (c[1] >= 0) ? -0.5 * (c[1] + sq) : -0.5 * (c[1] - sq);
        double r0 = q, r1 = (q != 0.0) ? c[0] / q : 0.0;
        if (r0 > r1) { double t = r0; r0 = r1; r1 = t; }
        roots[0] = r0; roots[1] = r1;
        return 2;
    }
    /* critical points from the derivative, then bracketed search */
    double dc[4];
    for (int i = 1; i <= deg; ++i) dc[i - 1] = c[i] * i;
    double crit[4];
    int nc = real_roots(dc, deg - 1, crit);
    double bound = 0;
    for (int i = 0; i < deg; ++i) if (fabs(c[i]) > bound) bound = fabs(c[i]);
    bound += 1.0;
    double pts[6];
    int np = 0;
    pts[np++] = -bound;
    for (int i = 0; i < nc; ++i) if (crit[i] > -bound && crit[i] < bound) pts[np++] = crit[i];
    pts[np++] = bound;
    int nr = 0;
    double fprev = peval(c, deg, pts[0]);
    for (int k = 1; k < np; ++k) {
        double f = peval(c, deg, pts[k]);
        if (f == 0.0) { roots[nr++] = pts[k]; }
        else if (fprev != 0.0 && ((f < 0) != (fprev < 0))) roots[nr++] = bracket_root(c, dc, deg, pts[k - 1], pts[k], fprev);
        fprev = f;
    }
    return nr;
}

/* ================================================================ P3P (Gao) */

typedef struct { double fx, fy, cx, cy, ifx, ify, cx_fx, cy_fx; } camk_t;

static void camk_init(camk_t* k, const double* K)
{
    k->fx = K[0]; k->fy = K[4]; k->cx = K[2]; k->cy = K[5];
    k->ifx = 1.0 / k->fx; k->ify = 1.0 / k->fy;
    k->cx_fx = k->cx / k->fx; k->cy_fx = k->cy / k->fy;
}

/* Horn's closed-form absolute orientation (unit quaternion = top eigenvector of N). */
static void jacobi_eig4(double* S, double* ev, double* U)
{
    for (int i = 0; i < 16; ++i) U[i] = (i % 5 == 0) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 50; ++sweep) {
        double off = 0;
        for (int i = 0; i < 4; ++i) for (int j = i + 1; j < 4; ++j) off += S[i * 4 + j] * S[i * 4 + j];
        if (off < 1e-300) break;
        for (int p = 0; p < 3; ++p) {
            for (int q = p + 1; q < 4; ++q) {
                double apq = S[p * 4 + q];
                if (apq == 0.0) continue;
                double theta = (S[q * 4 + q] - S[p * 4 + p]) / (2.0 * apq);
                double t = 1.0 / (fabs(theta) + sqrt(theta * theta + 1.0));
                if (theta < 0) t = -t;
                double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < 4; ++k) {
                    double skp = S[k * 4 + p], skq = S[k * 4 + q];
                    S[k * 4 + p] = c * skp - s * skq;
                    S[k * 4 + q] = s * skp + c * skq;
                }
                for (int k = 0; k < 4; ++k) {
                    double spk = S[p * 4 + k], sqk = S[q * 4 + k];
                    S[p * 4 + k] = c * spk - s * sqk;
                    S[q * 4 + k] = s * spk + c * sqk;
                }
                for (int k = 0; k < 4; ++k) {
                    double ukp = U[k * 4 + p], ukq = U[k * 4 + q];
                    U[k * 4 + p] = c * ukp - s * ukq;
                    U[k * 4 + q] = s * ukp + c * ukq;
                }
            }
        }
    }
    for (int i = 0; i < 4; ++i) ev[i] = S[i * 4 + i];
}

static void align_horn(const double M[3][3], const double P[3][3], double* R, double* T)
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
    int ib = 0;
    for (int i = 1; i < 4; ++i) if (ev[i] > ev[ib]) ib = i;
    double q0 = U[0 * 4 + ib], q1 = U[1 * 4 + ib], q2 = U[2 * 4 + ib], q3 = U[3 * 4 + ib];
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

/* Gao P3P: lengths along the three unit bearing rays.  Quartic in x = |C P0| / |C P2|:
 * N(x)^2 - b r x N(x) (p - r x) - b Q(x) (p - r x)^2 = 0, y = N(x) / (b (p - r x)),
 * N = (1-a-b) x^2 + (a-1) q x + (1-a+b),  Q = (1-b) x^2 - q x + 1. */
static int p3p_lengths(double L[4][3], const double d[3], const double cs[3])
{
    double p = cs[0] * 2, q = cs[1] * 2, r = cs[2] * 2;
    double inv_d22 = 1. / (d[2] * d[2]);
    double a = inv_d22 * (d[0] * d[0]);
    double b = inv_d22 * (d[1] * d[1]);
    if (p * p + q * q + r * r - p * q * r - 1 == 0) return 0;
    double n2 = 1 - a - b, n1 = (a - 1) * q, n0 = 1 - a + b;
    double A = n2 * n2 - a * b * r * r;
    if (A == 0) return 0;
    /* polynomial pieces, ascending coefficients */
    double Nn[3] = {n0, n1, n2};
    double NN[5] = {0};
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) NN[i + j] += Nn[i] * Nn[j];
    double Lp[2] = {p, -r};                  /* p - r x */
    double xLp[3] = {0, p, -r};              /* x (p - r x) */
    double LL[3] = {p * p, -2 * p * r, r * r};
    double Qq[3] = {1, -q, 1 - b};
    double c[5] = {0};
    for (int i = 0; i < 5; ++i) c[i] = NN[i];
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) if (i + j < 5) c[i + j] -= b * r * Nn[i] * xLp[j];
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) c[i + j] -= b * Qq[i] * LL[j];
    (void)Lp;
    double xs[4];
    int nr = real_roots(c, 4, xs);
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

/* pixel (float) -> normalised float32 (undistortPoints, zero distortion) -> pixel double */
static void p3p_reproject_input(const camk_t* k, double u, double v, double* uo, double* vo)
{
    float un = (float)((u - k->cx) * k->ifx);
    float vn = (float)((v - k->cy) * k->ify);
    *uo = (double)un * k->fx + k->cx;
    *vo = (double)vn * k->fy + k->cy;
}

/* 4-point P3P as solvePnP(SOLVEPNP_P3P): solve with points 0..2, pick by point 3. */
static int p3p_solve4(const camk_t* k, const double* obj, const double* img_px, double* Rb,
                      double* tb)
{
    double mu[4], mv[4], mk[3];
    for (int i = 0; i < 4; ++i) {
        double u, v;
        p3p_reproject_input(k, img_px[2 * i], img_px[2 * i + 1], &u, &v);
        mu[i] = k->ifx * u - k->cx_fx;
        mv[i] = k->ify * v - k->cy_fx;
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
            memcpy(Rb, R, sizeof R);
            memcpy(tb, T, sizeof T);
        }
    }
    return best >= 0;
}

int vo_o_p3p(const double* K, const double* obj4, const double* img4, double* R, double* t)
{
    camk_t k;
    camk_init(&k, K);
    return p3p_solve4(&k, obj4, img4, R, t);
}

/* ================================================================ EPnP */

/* deterministic sum over n items of K-vectors: item i -> partial (i % 64), then a
 * pairwise tree 32,16,...,1.  contrib(i, out[K]) supplies item i's vector. */
typedef void (*contrib_fn)(const void* ctx, int i, double* out);

static void det_sum(const void* ctx, contrib_fn f, int n, int K, double* out)
{
    double* part = (double*)calloc((size_t)NPART * K, sizeof(double));
    double tmp[160];
    for (int i = 0; i < n; ++i) {
        f(ctx, i, tmp);
        double* pp = part + (size_t)(i % NPART) * K;
        for (int k = 0; k < K; ++k) pp[k] += tmp[k];
    }
    for (int s = NPART / 2; s >= 1; s >>= 1)
        for (int t = 0; t < s; ++t)
            for (int k = 0; k < K; ++k) part[(size_t)t * K + k] += part[(size_t)(t + s) * K + k];
    memcpy(out, part, sizeof(double) * K);
    free(part);
}

typedef struct {
    int n;
    double fu, fv, uc, vc;
    const double* pws;   /* n x 3 */
    const double* us;    /* n x 2 (pixels) */
    double cws[4][3], ccs[4][3];
    double* alphas;      /* n x 4 */
    double* pcs;         /* n x 3 */
} epnp_t;

static void c_pw(const void* c, int i, double* o)
{
    const epnp_t* e = (const epnp_t*)c;
    o[0] = e->pws[3 * i]; o[1] = e->pws[3 * i + 1]; o[2] = e->pws[3 * i + 2];
}
static void c_pwcov(const void* c, int i, double* o)
{
    const epnp_t* e = (const epnp_t*)c;
    double d[3];
    for (int j = 0; j < 3; ++j) d[j] = e->pws[3 * i + j] - e->cws[0][j];
    for (int a = 0; a < 3; ++a) for (int b = 0; b < 3; ++b) o[a * 3 + b] = d[a] * d[b];
}
static void c_mtm(const void* c, int i, double* o)
{
    const epnp_t* e = (const epnp_t*)c;
    double M1[12], M2[12];
    const double* as = e->alphas + 4 * i;
    double u = e->us[2 * i], v = e->us[2 * i + 1];
    for (int k = 0; k < 4; ++k) {
        M1[3 * k] = as[k] * e->fu; M1[3 * k + 1] = 0.0; M1[3 * k + 2] = as[k] * (e->uc - u);
        M2[3 * k] = 0.0; M2[3 * k + 1] = as[k] * e->fv; M2[3 * k + 2] = as[k] * (e->vc - v);
    }
    /* upper triangle, 78 entries */
    int q = 0;
    for (int a = 0; a < 12; ++a) for (int b = a; b < 12; ++b) o[q++] = M1[a] * M1[b] + M2[a] * M2[b];
}
static void c_pc(const void* c, int i, double* o)
{
    const epnp_t* e = (const epnp_t*)c;
    o[0] = e->pcs[3 * i]; o[1] = e->pcs[3 * i + 1]; o[2] = e->pcs[3 * i + 2];
}
typedef struct { const epnp_t* e; double pc0[3], pw0[3]; } abt_ctx;
static void c_abt(const void* c, int i, double* o)
{
    const abt_ctx* a = (const abt_ctx*)c;
    for (int j = 0; j < 3; ++j)
        for (int k = 0; k < 3; ++k)
            o[j * 3 + k] = (a->e->pcs[3 * i + j] - a->pc0[j]) * (a->e->pws[3 * i + k] - a->pw0[k]);
}
typedef struct { const epnp_t* e; const double* R; const double* t; } rep_ctx;
static void c_rep(const void* c, int i, double* o)
{
    const rep_ctx* r = (const rep_ctx*)c;
    const double* pw = r->e->pws + 3 * i;
    const double* R = r->R;
    double Xc = R[0] * pw[0] + R[1] * pw[1] + R[2] * pw[2] + r->t[0];
    double Yc = R[3] * pw[0] + R[4] * pw[1] + R[5] * pw[2] + r->t[1];
    double inv_Zc = 1.0 / (R[6] * pw[0] + R[7] * pw[1] + R[8] * pw[2] + r->t[2]);
    double ue = r->e->uc + r->e->fu * Xc * inv_Zc;
    double ve = r->e->vc + r->e->fv * Yc * inv_Zc;
    double u = r->e->us[2 * i], v = r->e->us[2 * i + 1];
    o[0] = sqrt((u - ue) * (u - ue) + (v - ve) * (v - ve));
}

static const int PAIR_A[6] = {0, 0, 0, 1, 1, 2};
static const int PAIR_B[6] = {1, 2, 3, 2, 3, 3};

static void epnp_L6x10(const double* V12, double* L)
{
    /* v[i] = singular vector of the (i)-th smallest singular value: V column 11-i */
    double dv[4][6][3];
    for (int i = 0; i < 4; ++i) {
        int col = 11 - i;
        for (int j = 0; j < 6; ++j) {
            int a = PAIR_A[j], b = PAIR_B[j];
            for (int k = 0; k < 3; ++k) dv[i][j][k] = V12[(3 * a + k) * 12 + col] - V12[(3 * b + k) * 12 + col];
        }
    }
#define DOT3(p, q) ((p)[0] * (q)[0] + (p)[1] * (q)[1] + (p)[2] * (q)[2])
    for (int i = 0; i < 6; ++i) {
        double* row = L + 10 * i;
        row[0] = DOT3(dv[0][i], dv[0][i]);
        row[1] = 2.0 * DOT3(dv[0][i], dv[1][i]);
        row[2] = DOT3(dv[1][i], dv[1][i]);
        row[3] = 2.0 * DOT3(dv[0][i], dv[2][i]);
        row[4] = 2.0 * DOT3(dv[1][i], dv[2][i]);
        row[5] = DOT3(dv[2][i], dv[2][i]);
        row[6] = 2.0 * DOT3(dv[0][i], dv[3][i]);
        row[7] = 2.0 * DOT3(dv[1][i], dv[3][i]);
        row[8] = 2.0 * DOT3(dv[2][i], dv[3][i]);
        row[9] = DOT3(dv[3][i], dv[3][i]);
    }
}

static void qr_lsq(double* A, int m, int n, double* b, double* x)
{
    /* Householder QR least squares (m >= n) */
    for (int k = 0; k < n; ++k) {
        double nrm = 0;
        for (int i = k; i < m; ++i) nrm += A[i * n + k] * A[i * n + k];
        nrm = sqrt(nrm);
        if (nrm == 0) continue;
        double alpha = A[k * n + k] > 0 ? -nrm : nrm;
        double v[16];
        for (int i = k; i < m; ++i) v[i] = A[i * n + k];
        v[k] -= alpha;
        double vn = 0;
        for (int i = k; i < m; ++i) vn += v[i] * v[i];
        if (vn == 0) continue;
        for (int j = k; j < n; ++j) {
            double s = 0;
            for (int i = k; i < m; ++i) s += v[i] * A[i * n + j];
            s = 2.0 * s / vn;
            for (int i = k; i < m; ++i) A[i * n + j] -= s * v[i];
        }
        double s = 0;
        for (int i = k; i < m; ++i) s += v[i] * b[i];
        s = 2.0 * s / vn;
        for (int i = k; i < m; ++i) b[i] -= s * v[i];
    }
    for (int k = n - 1; k >= 0; --k) {
        double s = b[k];
        for (int j = k + 1; j < n; ++j) s -= A[k * n + j] * x[j];
        x[k] = (A[k * n + k] != 0) ? s / A[k * n + k] : 0.0;
    }
}

static void epnp_gauss_newton(const double* L, const double* rho, double* betas)
{
    for (int it = 0; it < 5; ++it) {
        double A[24], b[6], x[4];
        for (int i = 0; i < 6; ++i) {
            const double* rL = L + i * 10;
            double* rA = A + i * 4;
            rA[0] = 2 * rL[0] * betas[0] + rL[1] * betas[1] + rL[3] * betas[2] + rL[6] * betas[3];
            rA[1] = rL[1] * betas[0] + 2 * rL[2] * betas[1] + rL[4] * betas[2] + rL[7] * betas[3];
            rA[2] = rL[3] * betas[0] + rL[4] * betas[1] + 2 * rL[5] * betas[2] + rL[8] * betas[3];
            rA[3] = rL[6] * betas[0] + rL[7] * betas[1] + rL[8] * betas[2] + 2 * rL[9] * betas[3];
            b[i] = rho[i] - (rL[0] * betas[0] * betas[0] + rL[1] * betas[0] * betas[1] +
                             rL[2] * betas[1] * betas[1] + rL[3] * betas[0] * betas[2] +
                             rL[4] * betas[1] * betas[2] + rL[5] * betas[2] * betas[2] +
                             rL[6] * betas[0] * betas[3] + rL[7] * betas[1] * betas[3] +
                             rL[8] * betas[2] * betas[3] + rL[9] * betas[3] * betas[3]);
        }
        qr_lsq(A, 6, 4, b, x);
        for (int i = 0; i < 4; ++i) betas[i] += x[i];
    }
}

static double epnp_R_and_t(epnp_t* e, const double* V12, const double* betas, double* R, double* t)
{
    for (int j = 0; j < 4; ++j) for (int k = 0; k < 3; ++k) e->ccs[j][k] = 0;
    for (int i = 0; i < 4; ++i) {
        int col = 11 - i;
        for (int j = 0; j < 4; ++j)
            for (int k = 0; k < 3; ++k) e->ccs[j][k] += betas[i] * V12[(3 * j + k) * 12 + col];
    }
    for (int i = 0; i < e->n; ++i) {
        const double* a = e->alphas + 4 * i;
        for (int j = 0; j < 3; ++j)
            e->pcs[3 * i + j] = a[0] * e->ccs[0][j] + a[1] * e->ccs[1][j] + a[2] * e->ccs[2][j] + a[3] * e->ccs[3][j];
    }
    if (e->pcs[2] < 0.0) {
        for (int j = 0; j < 4; ++j) for (int k = 0; k < 3; ++k) e->ccs[j][k] = -e->ccs[j][k];
        for (int i = 0; i < 3 * e->n; ++i) e->pcs[i] = -e->pcs[i];
    }
    abt_ctx ac;
    ac.e = e;
    double s3[3];
    det_sum(e, c_pc, e->n, 3, s3);
    for (int j = 0; j < 3; ++j) ac.pc0[j] = s3[j] / e->n;
    det_sum(e, c_pw, e->n, 3, s3);
    for (int j = 0; j < 3; ++j) ac.pw0[j] = s3[j] / e->n;
    double abt[9], w[3], V[9];
    det_sum(&ac, c_abt, e->n, 9, abt);
    svd_jacobi(abt, 3, 3, w, V);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            R[i * 3 + j] = abt[i * 3 + 0] * V[j * 3 + 0] + abt[i * 3 + 1] * V[j * 3 + 1] + abt[i * 3 + 2] * V[j * 3 + 2];
    if (det3(R) < 0) { R[6] = -R[6]; R[7] = -R[7]; R[8] = -R[8]; }
    for (int i = 0; i < 3; ++i) t[i] = ac.pc0[i] - (R[i * 3] * ac.pw0[0] + R[i * 3 + 1] * ac.pw0[1] + R[i * 3 + 2] * ac.pw0[2]);
    rep_ctx rc = {e, R, t};
    double sum;
    det_sum(&rc, c_rep, e->n, 1, &sum);
    return sum / e->n;
}

int vo_o_epnp(const double* K, const double* obj, const double* img, int n, double* R, double* t)
{
    if (n < 4) return 0;
    epnp_t e;
    memset(&e, 0, sizeof e);
    e.n = n;
    e.fu = K[0]; e.fv = K[4]; e.uc = K[2]; e.vc = K[5];
    e.pws = obj;
    e.us = img;
    e.alphas = (double*)malloc(sizeof(double) * 4 * n);
    e.pcs = (double*)malloc(sizeof(double) * 3 * n);
    /* control points: centroid + principal axes */
    double s3[3];
    det_sum(&e, c_pw, n, 3, s3);
    for (int j = 0; j < 3; ++j) e.cws[0][j] = s3[j] / n;
    double cov[9], dc[3], Vc[9];
    det_sum(&e, c_pwcov, n, 9, cov);
    svd_jacobi(cov, 3, 3, dc, Vc);        /* cov holds U columns (= principal axes) */
    for (int i = 1; i < 4; ++i) {
        double k = sqrt(dc[i - 1] / n);
        for (int j = 0; j < 3; ++j) e.cws[i][j] = e.cws[0][j] + k * cov[j * 3 + (i - 1)];
    }
    /* barycentric coordinates: CC columns = cws[1..3] - cws[0]; pseudo-inverse via SVD */
    double CC[9], w[3], V[9], CCi[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 1; j < 4; ++j) CC[3 * i + j - 1] = e.cws[j][i] - e.cws[0][i];
    svd_jacobi(CC, 3, 3, w, V);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0;
            for (int k = 0; k < 3; ++k) if (w[k] > DBL_EPSILON * w[0] * 3) s += V[i * 3 + k] * CC[j * 3 + k] / w[k];
            CCi[i * 3 + j] = s;
        }
    for (int i = 0; i < n; ++i) {
        const double* pi = obj + 3 * i;
        double* a = e.alphas + 4 * i;
        for (int j = 0; j < 3; ++j)
            a[1 + j] = CCi[3 * j] * (pi[0] - e.cws[0][0]) + CCi[3 * j + 1] * (pi[1] - e.cws[0][1]) +
                       CCi[3 * j + 2] * (pi[2] - e.cws[0][2]);
        a[0] = 1.0 - a[1] - a[2] - a[3];
    }
    double up[78], MtM[144], dM[12], V12[144];
    det_sum(&e, c_mtm, n, 78, up);
    int q = 0;
    for (int a = 0; a < 12; ++a) for (int b = a; b < 12; ++b) { MtM[a * 12 + b] = MtM[b * 12 + a] = up[q++]; }
    svd_jacobi_rr(MtM, 12, 12, dM, V12);
    double L[60], rho[6];
    epnp_L6x10(V12, L);
    for (int j = 0; j < 6; ++j) {
        const double* p = e.cws[PAIR_A[j]];
        const double* r = e.cws[PAIR_B[j]];
        rho[j] = (p[0] - r[0]) * (p[0] - r[0]) + (p[1] - r[1]) * (p[1] - r[1]) + (p[2] - r[2]) * (p[2] - r[2]);
    }
    double betas[4][4], rep[4], Rs[4][9], ts[4][3];
    {   /* approx 1: columns 0,1,3,6 */
        double A[24], b4[4];
        static const int cols[4] = {0, 1, 3, 6};
        for (int i = 0; i < 6; ++i) for (int j = 0; j < 4; ++j) A[i * 4 + j] = L[i * 10 + cols[j]];
        lsq_svd(A, 6, 4, rho, b4);
        double* B = betas[1];
        if (b4[0] < 0) {
            B[0] = sqrt(-b4[0]); B[1] = -b4[1] / B[0]; B[2] = -b4[2] / B[0]; B[3] = -b4[3] / B[0];
        } else {
            B[0] = sqrt(b4[0]); B[1] = b4[1] / B[0]; B[2] = b4[2] / B[0]; B[3] = b4[3] / B[0];
        }
        epnp_gauss_newton(L, rho, B);
        rep[1] = epnp_R_and_t(&e, V12, B, Rs[1], ts[1]);
    }
    {   /* approx 2: columns 0,1,2 */
        double A[18], b3[3];
        for (int i = 0; i < 6; ++i) for (int j = 0; j < 3; ++j) A[i * 3 + j] = L[i * 10 + j];
        lsq_svd(A, 6, 3, rho, b3);
        double* B = betas[2];
        if (b3[0] < 0) { B[0] = sqrt(-b3[0]); B[1] = (b3[2] < 0) ? sqrt(-b3[2]) : 0.0; }
        else { B[0] = sqrt(b3[0]); B[1] = (b3[2] > 0) ? sqrt(b3[2]) : 0.0; }
        if (b3[1] < 0) B[0] = -B[0];
        B[2] = 0.0; B[3] = 0.0;
        epnp_gauss_newton(L, rho, B);
        rep[2] = epnp_R_and_t(&e, V12, B, Rs[2], ts[2]);
    }
    {   /* approx 3: columns 0..4 */
        double A[30], b5[5];
        for (int i = 0; i < 6; ++i) for (int j = 0; j < 5; ++j) A[i * 5 + j] = L[i * 10 + j];
        lsq_svd(A, 6, 5, rho, b5);
        double* B = betas[3];
        if (b5[0] < 0) { B[0] = sqrt(-b5[0]); B[1] = (b5[2] < 0) ? sqrt(-b5[2]) : 0.0; }
        else { B[0] = sqrt(b5[0]); B[1] = (b5[2] > 0) ? sqrt(b5[2]) : 0.0; }
        if (b5[1] < 0) B[0] = -B[0];
        B[2] = b5[3] / B[0]; B[3] = 0.0;
        epnp_gauss_newton(L, rho, B);
        rep[3] = epnp_R_and_t(&e, V12, B, Rs[3], ts[3]);
    }
    int N = 1;
    if (rep[2] < rep[1]) N = 2;
    if (rep[3] < rep[N]) N = 3;
    memcpy(R, Rs[N], sizeof(double) * 9);
    memcpy(t, ts[N], sizeof(double) * 3);
    free(e.alphas);
    free(e.pcs);
    return 1;
}

/* ================================================================ RANSAC core */

static int ransac_update_niters(double p, double ep, int model_points, int max_iters)
{
    p = p < 0 ? 0 : (p > 1 ? 1 : p);
    ep = ep < 0 ? 0 : (ep > 1 ? 1 : ep);
    double num = 1. - p > DBL_MIN ? 1. - p : DBL_MIN;
    double denom = 1. - vcr_powi(1. - ep, model_points);
    if (denom < DBL_MIN) return 0;
    num = vcr_log(num);
    denom = vcr_log(denom);
    return (denom >= 0 || -num >= max_iters * (-denom)) ? max_iters : (int)lrint(num / denom);
}

/* getSubset: draw model_points distinct indices in [0, count) */
static void get_subset(uint64_t* rng, int count, int mp, int* idx)
{
    for (int i = 0; i < mp; ++i) {
        for (;;) {
            int v = (int)(vo_o_rng_next(rng) % (uint32_t)count);
            int j;
            for (j = 0; j < i; ++j) if (v == idx[j]) break;
            idx[i] = v;
            if (j == i) break;
        }
    }
}

/* projectPoints (zero distortion) -> float, squared error in float */
static inline float pnp_err(const double* R, const double* t, const camk_t* k, const float* X,
                            const float* x)
{
    double Xd = X[0], Yd = X[1], Zd = X[2];
    double xx = R[0] * Xd + R[1] * Yd + R[2] * Zd + t[0];
    double yy = R[3] * Xd + R[4] * Yd + R[5] * Zd + t[1];
    double zz = R[6] * Xd + R[7] * Yd + R[8] * Zd + t[2];
    zz = zz != 0.0 ? 1. / zz : 1;
    xx *= zz;
    yy *= zz;
    float pu = (float)(xx * k->fx + k->cx);
    float pv = (float)(yy * k->fy + k->cy);
    float du = x[0] - pu, dv = x[1] - pv;
    return du * du + dv * dv;
}

int vo_o_pnp_ransac_p3p(const float* obj, const float* img, int n, const double* K,
                        int iterations, double reproj_err, double confidence,
                        double* rvec, double* tvec, int32_t* inliers, int* n_inl,
                        int* success, int* iters_out)
{
    if (!obj || !img || !K || !rvec || !tvec || !n_inl || !success) return VO_O_EARG;
    *success = 0;
    *n_inl = 0;
    if (iters_out) *iters_out = 0;
    if (n < 4) return VO_O_EARG;
    camk_t k;
    camk_init(&k, K);
    const int mp = 4;
    double bestR[9], bestt[3];
    int best_count = 0;
    uint8_t* mask = (uint8_t*)malloc(n);
    float thr = (float)(reproj_err * reproj_err);
    if (n == mp) {
        double o[12], im[8];
        for (int i = 0; i < 12; ++i) o[i] = obj[i];
        for (int i = 0; i < 8; ++i) im[i] = img[i];
        if (!p3p_solve4(&k, o, im, bestR, bestt)) { free(mask); return VO_O_OK; }
        vo_o_rodrigues_m2v(bestR, rvec);
        memcpy(tvec, bestt, sizeof bestt);
        for (int i = 0; i < n; ++i) if (inliers) inliers[i] = i;
        *n_inl = n;
        *success = 1;
        free(mask);
        return VO_O_OK;
    }
    uint64_t rng = ~0ULL;
    int niters = iterations > 1 ? iterations : 1;
    int iter;
    for (iter = 0; iter < niters; ++iter) {
        int idx[4];
        get_subset(&rng, n, mp, idx);
        double o[12], im[8], R[9], t[3];
        for (int j = 0; j < 4; ++j) {
            o[3 * j] = obj[3 * idx[j]]; o[3 * j + 1] = obj[3 * idx[j] + 1]; o[3 * j + 2] = obj[3 * idx[j] + 2];
            im[2 * j] = img[2 * idx[j]]; im[2 * j + 1] = img[2 * idx[j] + 1];
        }
        if (!p3p_solve4(&k, o, im, R, t)) continue;
        int good = 0;
        for (int i = 0; i < n; ++i) good += pnp_err(R, t, &k, obj + 3 * i, img + 2 * i) <= thr;
        if (good > (best_count > mp - 1 ? best_count : mp - 1)) {
            best_count = good;
            memcpy(bestR, R, sizeof R);
            memcpy(bestt, t, sizeof t);
            niters = ransac_update_niters(confidence, (double)(n - good) / n, mp, niters);
        }
    }
    if (iters_out) *iters_out = iter;
    if (best_count <= 0) { free(mask); return VO_O_OK; }
    int m = 0;
    for (int i = 0; i < n; ++i) {
        mask[i] = pnp_err(bestR, bestt, &k, obj + 3 * i, img + 2 * i) <= thr;
        m += mask[i];
    }
    /* final EPnP refit on inliers (solvePnP(..., SOLVEPNP_EPNP)) */
    double* o = (double*)malloc(sizeof(double) * 3 * m);
    double* im = (double*)malloc(sizeof(double) * 2 * m);
    int q = 0;
    for (int i = 0; i < n; ++i) {
        if (!mask[i]) continue;
        o[3 * q] = obj[3 * i]; o[3 * q + 1] = obj[3 * i + 1]; o[3 * q + 2] = obj[3 * i + 2];
        /* EPnP receives double points: undistortPoints (double) then x*fx + cx */
        double un = ((double)img[2 * i] - k.cx) * k.ifx, vn = ((double)img[2 * i + 1] - k.cy) * k.ify;
        im[2 * q] = un * k.fx + k.cx; im[2 * q + 1] = vn * k.fy + k.cy;
        if (inliers) inliers[q] = i;
        ++q;
    }
    double R[9], t[3];
    int ok = vo_o_epnp(K, o, im, m, R, t);
    free(o);
    free(im);
    free(mask);
    if (!ok) {
        vo_o_rodrigues_m2v(bestR, rvec);
        memcpy(tvec, bestt, sizeof bestt);
        return VO_O_OK;
    }
    vo_o_rodrigues_m2v(R, rvec);
    memcpy(tvec, t, sizeof t);
    *n_inl = m;
    *success = 1;
    return VO_O_OK;
}

/* ================================================================ five-point */

/* monomials of degree <= 3 in (x,y,z), column order of the 10x20 system */
static const int MONO[20][3] = {
    {3, 0, 0}, {0, 3, 0}, {2, 1, 0}, {1, 2, 0}, {2, 0, 1}, {2, 0, 0}, {0, 2, 1}, {0, 2, 0},
    {1, 1, 1}, {1, 1, 0}, {1, 0, 2}, {1, 0, 1}, {1, 0, 0}, {0, 1, 2}, {0, 1, 1}, {0, 1, 0},
    {0, 0, 3}, {0, 0, 2}, {0, 0, 1}, {0, 0, 0}};

/* polynomial in x,y,z of degree <= 3 stored by MONO index (20 coefficients); products
 * accumulate term pairs in (i, j) MONO order so CPU and GPU round identically */
typedef struct { double c[20]; } poly3_t;

static int g_prod[20][20];     /* MONO index of MONO[i]*MONO[j], or -1 if degree > 3 */
static int g_prod_init = 0;

static void prod_init(void)
{
    if (g_prod_init) return;
    for (int i = 0; i < 20; ++i)
        for (int j = 0; j < 20; ++j) {
            int a = MONO[i][0] + MONO[j][0], b = MONO[i][1] + MONO[j][1], c = MONO[i][2] + MONO[j][2];
            g_prod[i][j] = -1;
            if (a + b + c > 3) continue;
            for (int k = 0; k < 20; ++k)
                if (MONO[k][0] == a && MONO[k][1] == b && MONO[k][2] == c) g_prod[i][j] = k;
        }
    g_prod_init = 1;
}

static void p_zero(poly3_t* p) { memset(p, 0, sizeof *p); }
static void p_mul(const poly3_t* a, const poly3_t* b, poly3_t* out)
{
    poly3_t r;
    p_zero(&r);
    for (int i = 0; i < 20; ++i) {
        if (a->c[i] == 0.0) continue;
        for (int j = 0; j < 20; ++j) {
            if (b->c[j] == 0.0) continue;
            int k = g_prod[i][j];
            if (k < 0) continue;
            r.c[k] += a->c[i] * b->c[j];
        }
    }
    *out = r;
}
static void p_axpy(double s, const poly3_t* a, poly3_t* y)
{
    for (int i = 0; i < 20; ++i) y->c[i] += s * a->c[i];
}

/* Weierstrass / Durand-Kerner as in cv::solvePoly; c ascending (deg n), roots re/im */
typedef struct { double re, im; } cplx;
static cplx c_mul(cplx a, cplx b) { cplx r = {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; return r; }
static cplx c_sub(cplx a, cplx b) { cplx r = {a.re - b.re, a.im - b.im}; return r; }
static cplx c_add(cplx a, cplx b) { cplx r = {a.re + b.re, a.im + b.im}; return r; }
static cplx c_div(cplx a, cplx b)
{
    double t = 1. / (b.re * b.re + b.im * b.im);
    cplx r = {(a.re * b.re + a.im * b.im) * t, (-a.re * b.im + a.im * b.re) * t};
    return r;
}

static int solve_poly(const double* c_in, int n0, cplx* roots)
{
    cplx co[11];
    for (int i = 0; i <= n0; ++i) { co[i].re = c_in[i]; co[i].im = 0; }
    int n = n0;
    for (; n > 1; --n) if (fabs(co[n].re) + fabs(co[n].im) > DBL_EPSILON) break;
    cplx p = {1, 0}, r = {1, 1};
    for (int i = 0; i < n; ++i) { roots[i] = p; p = c_mul(p, r); }
    for (int iter = 0; iter < 300; ++iter) {
        double maxDiff = 0;
        for (int i = 0; i < n; ++i) {
            p = roots[i];
            cplx num = co[n], denom = co[n];
            int same = 1;
            for (int j = 0; j < n; ++j) {
                num = c_add(c_mul(num, p), co[n - j - 1]);
                if (j != i) {
                    cplx d = c_sub(p, roots[j]);
                    if (d.re == 0 && d.im == 0) same++;
                    else denom = c_mul(denom, d);
                }
            }
            num = c_div(num, denom);
            (void)same;
            roots[i] = c_sub(p, num);
            double a = sqrt(num.re * num.re + num.im * num.im);
            if (a > maxDiff) maxDiff = a;
        }
        if (maxDiff <= 0) break;
    }
    for (int i = 0; i < n; ++i) if (fabs(roots[i].im) < 1e-100) roots[i].im = 0;
    return n;
}

static void null3(const double* B, double* v)
{
    double A[9], w[3], V[9];
    memcpy(A, B, sizeof A);
    svd_jacobi(A, 3, 3, w, V);
    v[0] = V[2]; v[1] = V[5]; v[2] = V[8];
}

int vo_o_five_point(const double* q1, const double* q2, double* E10)
{
    prod_init();
    /* Q (5 x 9): x2^T E x1 = 0 with e = vec(E) row-major */
    double Qt[9 * 5];   /* transpose, 9 x 5 */
    for (int i = 0; i < 5; ++i) {
        double x1 = q1[2 * i], y1 = q1[2 * i + 1], x2 = q2[2 * i], y2 = q2[2 * i + 1];
        double row[9] = {x1 * x2, y1 * x2, x2, x1 * y2, y1 * y2, y2, x1, y1, 1.0};
        for (int j = 0; j < 9; ++j) Qt[j * 5 + i] = row[j];
    }
    /* Householder QR of Qt (9x5); null space of Q = last 4 columns of the full orthogonal factor */
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
    double basis[4][9];
    for (int b = 0; b < 4; ++b) {
        double v[9] = {0};
        v[5 + b] = 1.0;
        for (int k = 4; k >= 0; --k) {
            if (hn[k] == 0) continue;
            double s = 0;
            for (int i = k; i < 9; ++i) s += H[k][i] * v[i];
            s = 2.0 * s / hn[k];
            for (int i = k; i < 9; ++i) v[i] -= s * H[k][i];
        }
        memcpy(basis[b], v, sizeof v);
    }
    /* E(x,y,z) = x X + y Y + z Z + W as linear polynomials */
    poly3_t Ep[9];
    for (int e = 0; e < 9; ++e) {
        p_zero(&Ep[e]);
        Ep[e].c[12] = basis[0][e];
        Ep[e].c[15] = basis[1][e];
        Ep[e].c[18] = basis[2][e];
        Ep[e].c[19] = basis[3][e];
    }
    poly3_t eqs[10];
    /* det(E) */
    {
        poly3_t t1, t2, acc;
        p_zero(&acc);
        int cof[3][4] = {{4, 8, 5, 7}, {3, 8, 5, 6}, {3, 7, 4, 6}};
        double sg[3] = {1, -1, 1};
        for (int c = 0; c < 3; ++c) {
            poly3_t m1, m2;
            p_mul(&Ep[cof[c][0]], &Ep[cof[c][1]], &m1);
            p_mul(&Ep[cof[c][2]], &Ep[cof[c][3]], &m2);
            p_axpy(-1.0, &m2, &m1);
            p_mul(&Ep[c], &m1, &t1);
            p_axpy(sg[c], &t1, &acc);
        }
        (void)t2;
        eqs[0] = acc;
    }
    /* 2 E E^T E - tr(E E^T) E */
    {
        poly3_t EEt[9];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                p_zero(&EEt[i * 3 + j]);
                for (int k = 0; k < 3; ++k) {
                    poly3_t m;
                    p_mul(&Ep[i * 3 + k], &Ep[j * 3 + k], &m);
                    p_axpy(1.0, &m, &EEt[i * 3 + j]);
                }
            }
        poly3_t tr;
        p_zero(&tr);
        p_axpy(1.0, &EEt[0], &tr);
        p_axpy(1.0, &EEt[4], &tr);
        p_axpy(1.0, &EEt[8], &tr);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                poly3_t acc, m;
                p_zero(&acc);
                for (int k = 0; k < 3; ++k) {
                    p_mul(&EEt[i * 3 + k], &Ep[k * 3 + j], &m);
                    p_axpy(2.0, &m, &acc);
                }
                p_mul(&tr, &Ep[i * 3 + j], &m);
                p_axpy(-1.0, &m, &acc);
                eqs[1 + i * 3 + j] = acc;
            }
    }
    double A[10 * 10], Bm[10 * 10];
    for (int r = 0; r < 10; ++r)
        for (int c = 0; c < 20; ++c) {
            double v = eqs[r].c[c];
            if (c < 10) A[r * 10 + c] = v; else Bm[r * 10 + (c - 10)] = v;
        }
    if (!gauss_solve(A, 10, Bm, 10)) return 0;
    /* B (3 x 13): rows <x2z> - z<x2>, <y2z> - z<y2>, <xyz> - z<xy> */
    double b[3][13];
    for (int i = 0; i < 3; ++i) {
        const double* g1 = Bm + (4 + 2 * i) * 10;
        const double* g2 = Bm + (5 + 2 * i) * 10;
        double r1[13] = {0}, r2[13] = {0};
        r1[1] = g1[0]; r1[2] = g1[1]; r1[3] = g1[2];
        r1[5] = g1[3]; r1[6] = g1[4]; r1[7] = g1[5];
        r1[9] = g1[6]; r1[10] = g1[7]; r1[11] = g1[8]; r1[12] = g1[9];
        r2[0] = g2[0]; r2[1] = g2[1]; r2[2] = g2[2];
        r2[4] = g2[3]; r2[5] = g2[4]; r2[6] = g2[5];
        r2[8] = g2[6]; r2[9] = g2[7]; r2[10] = g2[8]; r2[11] = g2[9];
        for (int k = 0; k < 13; ++k) b[i][k] = r1[k] - r2[k];
    }
    /* det of [[px_i(z), py_i(z), p1_i(z)]] : px,py cubic (coeffs z^3..z^0), p1 quartic */
    double P[3][3][5];   /* ascending in z */
    for (int i = 0; i < 3; ++i) {
        for (int k = 0; k < 5; ++k) P[i][0][k] = P[i][1][k] = P[i][2][k] = 0;
        for (int k = 0; k < 4; ++k) { P[i][0][3 - k] = b[i][k]; P[i][1][3 - k] = b[i][4 + k]; }
        for (int k = 0; k < 5; ++k) P[i][2][4 - k] = b[i][8 + k];
    }
    double coeffs[11] = {0};
    {
        static const int perm[6][3] = {{0, 1, 2}, {0, 2, 1}, {1, 0, 2}, {1, 2, 0}, {2, 0, 1}, {2, 1, 0}};
        static const double psign[6] = {1, -1, -1, 1, 1, -1};
        for (int s = 0; s < 6; ++s) {
            double t1[9] = {0}, t2[11] = {0};
            for (int a = 0; a < 5; ++a) for (int c = 0; c < 5; ++c)
                if (a + c < 9) t1[a + c] += P[0][perm[s][0]][a] * P[1][perm[s][1]][c];
            for (int a = 0; a < 9; ++a) for (int c = 0; c < 5; ++c)
                if (a + c < 11) t2[a + c] += t1[a] * P[2][perm[s][2]][c];
            for (int k = 0; k < 11; ++k) coeffs[k] += psign[s] * t2[k];
        }
    }
    cplx roots[10];
    int nroots = solve_poly(coeffs, 10, roots);
    int count = 0;
    for (int i = 0; i < nroots; ++i) {
        if (fabs(roots[i].im) > 1e-10) continue;
        double z1 = roots[i].re, z2 = z1 * z1, z3 = z2 * z1, z4 = z3 * z1;
        double Bz[9];
        for (int j = 0; j < 3; ++j) {
            const double* br = b[j];
            Bz[j * 3 + 0] = br[0] * z3 + br[1] * z2 + br[2] * z1 + br[3];
            Bz[j * 3 + 1] = br[4] * z3 + br[5] * z2 + br[6] * z1 + br[7];
            Bz[j * 3 + 2] = br[8] * z4 + br[9] * z3 + br[10] * z2 + br[11] * z1 + br[12];
        }
        double xy1[3];
        null3(Bz, xy1);
        if (fabs(xy1[2]) < 1e-10) continue;
        double x = xy1[0] / xy1[2], y = xy1[1] / xy1[2];
        double ev[9], nrm = 0;
        for (int e = 0; e < 9; ++e) {
            ev[e] = basis[0][e] * x + basis[1][e] * y + basis[2][e] * z1 + basis[3][e];
            nrm += ev[e] * ev[e];
        }
        nrm = sqrt(nrm);
        for (int e = 0; e < 9; ++e) E10[count * 9 + e] = ev[e] / nrm;
        ++count;
    }
    return count;
}

static inline float sampson_err(const double* E, double x1, double y1, double x2, double y2)
{
    double Ex1[3] = {E[0] * x1 + E[1] * y1 + E[2], E[3] * x1 + E[4] * y1 + E[5], E[6] * x1 + E[7] * y1 + E[8]};
    double Etx2[3] = {E[0] * x2 + E[3] * y2 + E[6], E[1] * x2 + E[4] * y2 + E[7], E[2] * x2 + E[5] * y2 + E[8]};
    double x2tEx1 = x2 * Ex1[0] + y2 * Ex1[1] + Ex1[2];
    double a = Ex1[0] * Ex1[0], b = Ex1[1] * Ex1[1], c = Etx2[0] * Etx2[0], d = Etx2[1] * Etx2[1];
    return (float)(x2tEx1 * x2tEx1 / (a + b + c + d));
}

int vo_o_find_essential(const float* p0, const float* p1, int n, const double* K, double prob,
                        double threshold, int max_iters, double* E, uint8_t* mask, int* n_models_out)
{
    if (!p0 || !p1 || !K || !E || n < 0) return VO_O_EARG;
    double fx = K[0], fy = K[4], cx = K[2], cy = K[5];
    double* q1 = (double*)malloc(sizeof(double) * 2 * (n > 0 ? n : 1));
    double* q2 = (double*)malloc(sizeof(double) * 2 * (n > 0 ? n : 1));
    for (int i = 0; i < n; ++i) {
        q1[2 * i] = ((double)p0[2 * i] - cx) / fx;
        q1[2 * i + 1] = ((double)p0[2 * i + 1] - cy) / fy;
        q2[2 * i] = ((double)p1[2 * i] - cx) / fx;
        q2[2 * i + 1] = ((double)p1[2 * i + 1] - cy) / fy;
    }
    threshold /= (fx + fy) / 2;
    float thr = (float)(threshold * threshold);
    const int mp = 5;
    int result = 0, total_models = 0;
    memset(E, 0, sizeof(double) * 9);
    if (n < mp) goto done;
    if (n == mp) {
        double E10[90];
        int nm = vo_o_five_point(q1, q2, E10);
        total_models = nm;
        if (nm > 0) {
            /* run(): count == modelPoints -> the whole model block, mask all ones.
               With several solutions OpenCV returns the stacked block; keep the first. */
            memcpy(E, E10, sizeof(double) * 9);
            if (mask) memset(mask, 1, n);
            result = 1;
        }
        goto done;
    }
    {
        uint64_t rng = ~0ULL;
        int niters = max_iters > 1 ? max_iters : 1;
        int best = 0;
        uint8_t* cur = (uint8_t*)malloc(n);
        for (int iter = 0; iter < niters; ++iter) {
            int idx[5];
            get_subset(&rng, n, mp, idx);
            double s1[10], s2[10], E10[90];
            for (int j = 0; j < 5; ++j) {
                s1[2 * j] = q1[2 * idx[j]]; s1[2 * j + 1] = q1[2 * idx[j] + 1];
                s2[2 * j] = q2[2 * idx[j]]; s2[2 * j + 1] = q2[2 * idx[j] + 1];
            }
            int nm = vo_o_five_point(s1, s2, E10);
            total_models += nm;
            for (int m = 0; m < nm; ++m) {
                const double* Em = E10 + 9 * m;
                int good = 0;
                for (int i = 0; i < n; ++i) {
                    cur[i] = sampson_err(Em, q1[2 * i], q1[2 * i + 1], q2[2 * i], q2[2 * i + 1]) <= thr;
                    good += cur[i];
                }
                if (good > (best > mp - 1 ? best : mp - 1)) {
                    best = good;
                    memcpy(E, Em, sizeof(double) * 9);
                    if (mask) memcpy(mask, cur, n);
                    niters = ransac_update_niters(prob, (double)(n - good) / n, mp, niters);
                }
            }
        }
        free(cur);
        result = best > 0;
    }
done:
    if (!result && mask && n > 0) memset(mask, 0, n);
    if (n_models_out) *n_models_out = total_models;
    free(q1);
    free(q2);
    return result ? VO_O_OK : VO_O_EFAIL;
}

int vo_o_recover_pose(const double* E, const float* p0, const float* p1, int n, const double* K,
                      double* R, double* t, uint8_t* mask, int* n_good)
{
    if (!E || !K || !R || !t || n < 0) return VO_O_EARG;
    double fx = K[0], fy = K[4], cx = K[2], cy = K[5];
    double* x1 = (double*)malloc(sizeof(double) * 2 * (n > 0 ? n : 1));
    double* x2 = (double*)malloc(sizeof(double) * 2 * (n > 0 ? n : 1));
    for (int i = 0; i < n; ++i) {
        x1[2 * i] = ((double)p0[2 * i] - cx) / fx;
        x1[2 * i + 1] = ((double)p0[2 * i + 1] - cy) / fy;
        x2[2 * i] = ((double)p1[2 * i] - cx) / fx;
        x2[2 * i + 1] = ((double)p1[2 * i + 1] - cy) / fy;
    }
    /* decomposeEssentialMat */
    double U[9], w[3], V[9];
    memcpy(U, E, sizeof U);
    svd_jacobi(U, 3, 3, w, V);
    if (det3(U) < 0) for (int i = 0; i < 9; ++i) U[i] = -U[i];
    if (det3(V) < 0) for (int i = 0; i < 9; ++i) V[i] = -V[i];   /* det(Vt) == det(V) */
    double W[9] = {0, 1, 0, -1, 0, 0, 0, 0, 1}, Wt[9] = {0, -1, 0, 1, 0, 0, 0, 0, 1};
    double Vt[9], UW[9], R1[9], R2[9], tt[3];
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) Vt[i * 3 + j] = V[j * 3 + i];
    matmul3(U, W, UW);
    matmul3(UW, Vt, R1);
    matmul3(U, Wt, UW);
    matmul3(UW, Vt, R2);
    for (int i = 0; i < 3; ++i) tt[i] = U[i * 3 + 2];
    const double dist = 50.0;
    double P0[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    double* Q = (double*)malloc(sizeof(double) * 4 * (n > 0 ? n : 1));
    uint8_t* masks = (uint8_t*)malloc((size_t)4 * (n > 0 ? n : 1));
    int good[4];
    for (int c = 0; c < 4; ++c) {
        const double* Rc = (c == 0 || c == 2) ? R1 : R2;
        double sg = (c < 2) ? 1.0 : -1.0;
        double P[12];
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) P[i * 4 + j] = Rc[i * 3 + j];
            P[i * 4 + 3] = sg * tt[i];
        }
        vo_o_triangulate_d(P0, P, x1, x2, n, Q);
        good[c] = 0;
        for (int i = 0; i < n; ++i) {
            double X = Q[i], Y = Q[n + i], Z = Q[2 * n + i], Wh = Q[3 * n + i];
            int m = (Z * Wh) > 0;
            X /= Wh; Y /= Wh; Z /= Wh;
            double W1 = Wh / Wh;
            m = m && (Z < dist);
            double z2 = P[8] * X + P[9] * Y + P[10] * Z + P[11] * W1;
            m = m && (z2 > 0);
            m = m && (z2 < dist);
            masks[(size_t)c * n + i] = (uint8_t)m;
            good[c] += m;
        }
    }
    int sel;
    if (good[0] >= good[1] && good[0] >= good[2] && good[0] >= good[3]) sel = 0;
    else if (good[1] >= good[0] && good[1] >= good[2] && good[1] >= good[3]) sel = 1;
    else if (good[2] >= good[0] && good[2] >= good[1] && good[2] >= good[3]) sel = 2;
    else sel = 3;
    memcpy(R, (sel == 0 || sel == 2) ? R1 : R2, sizeof(double) * 9);
    for (int i = 0; i < 3; ++i) t[i] = (sel < 2) ? tt[i] : -tt[i];
    if (mask) memcpy(mask, masks + (size_t)sel * n, n);
    if (n_good) *n_good = good[sel];
    free(Q);
    free(masks);
    free(x1);
    free(x2);
    return VO_O_OK;
}
