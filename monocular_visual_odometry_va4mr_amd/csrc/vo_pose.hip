// Pose-side kernels for gfx950: PnP-RANSAC (P3P hypotheses, wave-parallel scoring,
// OpenCV's sequential "first strictly better + adaptive niters" rule) with the EPnP
// refit, candidate triangulation with ordered append/compaction, and the feature-adding
// distance filter + step finish.
//
// Reference call sites: VisualOdometryPipeLine.py:107-206 (triangulate_landmarks incl.
// cv2.triangulatePoints :188), :248-268 (feature_adding filter), :338-373 (PnP step and
// bookkeeping).  fp64 geometry lives in vo_dgeom.h and mirrors oracle/vo_oracle_geom.c.
#include "vo_dgeom.h"

namespace {

using namespace vg;

#ifdef VO_PNP_PROF
__device__ long long g_pnpprof[32];
}  // namespace
// diagnostics build only (libvo_hip_pnpprof.so, tools/pnp_prof.py): block 0's phase timestamps
// of the last PnP launch (100 MHz wall clock)
extern "C" int vo_pnp_prof_read(long long* out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pnpprof), sizeof(long long) * 32) == hipSuccess ? 0 : -2;
}
namespace {
#define PNPPROF(i) do { if (threadIdx.x == 0 && blockIdx.x == 0) g_pnpprof[i] = wall_clock64(); } while (0)
#define PNPVAL(i, v) do { if (threadIdx.x == 0 && blockIdx.x == 0) g_pnpprof[i] = (v); } while (0)
#define PNPPROF_T(i, t) do { if (threadIdx.x == (t) && blockIdx.x == 0) g_pnpprof[i] = wall_clock64(); } while (0)
#else
#define PNPPROF_T(i, t) do { } while (0)
#define PNPPROF(i) do { } while (0)
#define PNPVAL(i, v) do { } while (0)
#endif

// ------------------------------------------------------------------ EPnP (block)
struct EpnpShared {
    double cws[4][3], ccs[4][3];
    double CCi[9];
    double V12[144];
    double L[60], rho[6];
    double betas[4][4], rep[4], Rs[4][9], ts[4][3];
    double tmp[80];
    double MtM[144], dM[12];
    double pc0[3], pw0[3];
    int flip;
};

// Sum over n items of K-vectors in the oracle's fixed order (lane = item % 64, then a
// shuffle tree 32..1).  Executed by wave 0; result in out[0..K) (LDS).
template <int K, class F>
VO_DEV void wave_det_sum(int n, F f, double* out)
{
    const int lane = lane_id();
    double acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = 0.0;
    for (int i = lane; i < n; i += 64) {
        double c[K];
        f(i, c);
#pragma unroll
        for (int k = 0; k < K; ++k) acc[k] += c[k];
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        double v = acc[k];
        for (int s = 32; s >= 1; s >>= 1) v += __shfl_down(v, s, 64);
        if (lane == 0) out[k] = v;
    }
}

// Householder least squares (the oracle's qr_lsq), sizes fixed at compile time so the
// working arrays stay in registers
template <int M, int N>
VO_DEV void qr_lsq(double* A, double* b, double* x)
{
#pragma unroll
    for (int k = 0; k < N; ++k) {
        double nrm = 0;
#pragma unroll
        for (int i = k; i < M; ++i) nrm += A[i * N + k] * A[i * N + k];
        nrm = sqrt(nrm);
        if (nrm == 0) continue;
        double alpha = A[k * N + k] > 0 ? -nrm : nrm;
        double v[M];
#pragma unroll
        for (int i = k; i < M; ++i) v[i] = A[i * N + k];
        v[k] -= alpha;
        double vn = 0;
#pragma unroll
        for (int i = k; i < M; ++i) vn += v[i] * v[i];
        if (vn == 0) continue;
#pragma unroll
        for (int j = k; j < N; ++j) {
            double s = 0;
#pragma unroll
            for (int i = k; i < M; ++i) s += v[i] * A[i * N + j];
            s = 2.0 * s / vn;
#pragma unroll
            for (int i = k; i < M; ++i) A[i * N + j] -= s * v[i];
        }
        double s = 0;
#pragma unroll
        for (int i = k; i < M; ++i) s += v[i] * b[i];
        s = 2.0 * s / vn;
#pragma unroll
        for (int i = k; i < M; ++i) b[i] -= s * v[i];
    }
#pragma unroll
    for (int k = N - 1; k >= 0; --k) {
        double s = b[k];
#pragma unroll
        for (int j = k + 1; j < N; ++j) s -= A[k * N + j] * x[j];
        x[k] = (A[k * N + k] != 0) ? s / A[k * N + k] : 0.0;
    }
}

VO_DEV void epnp_gauss_newton(const double* L, const double* rho, double* betas)
{
    for (int it = 0; it < 5; ++it) {
        double A[24], b[6], x[4];
#pragma unroll
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
        qr_lsq<6, 4>(A, b, x);
#pragma unroll
        for (int i = 0; i < 4; ++i) betas[i] += x[i];
    }
}

__constant__ int PAIR_A[6] = {0, 0, 0, 1, 1, 2};
__constant__ int PAIR_B[6] = {1, 2, 3, 2, 3, 3};

VO_DEV void epnp_L6x10(const double* V12, double* L)
{
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
#undef DOT3
}

// Entries [Q0, Q1) of the upper triangle of M^T M (row-major a <= b), summed in the order
// of wave_det_sum (item i -> lane i % 64, serial per lane, then the shuffle tree).
template <int Q0, int Q1>
VO_DEV void epnp_mtm_part(int n, const double* alphas, const double* us, double fu, double fv, double uc,
                          double vc, double* up)
{
    constexpr int K = Q1 - Q0;
    const int lane = lane_id();
    double acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = 0.0;
    for (int i = lane; i < n; i += 64) {
        double M1[12], M2[12];
        const double* as = alphas + 4 * i;
        const double u = us[2 * i], v = us[2 * i + 1];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            M1[3 * k] = as[k] * fu; M1[3 * k + 1] = 0.0; M1[3 * k + 2] = as[k] * (uc - u);
            M2[3 * k] = 0.0; M2[3 * k + 1] = as[k] * fv; M2[3 * k + 2] = as[k] * (vc - v);
        }
        int q = 0;
#pragma unroll
        for (int a = 0; a < 12; ++a)
#pragma unroll
            for (int b = a; b < 12; ++b, ++q)
                if (q >= Q0 && q < Q1) acc[q - Q0] += M1[a] * M1[b] + M2[a] * M2[b];
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        double v = acc[k];
        for (int s = 32; s >= 1; s >>= 1) v += __shfl_down(v, s, 64);
        if (lane == 0) up[Q0 + k] = v;
    }
}

// compute_R_and_t for approximation `a`, executed by one whole wave (the three
// approximations run on waves 0..2 at once).  The camera-frame points pcs are recomputed
// from alphas and ccs where needed instead of being stored (same products and sums; the
// sign flip negates ccs, which negates every pcs exactly).  S.pw0 is set by the caller.
VO_DEV void epnp_R_and_t_wave(EpnpShared& S, int a, const double* K, const double* pws, const double* us,
                              const double* alphas, int n)
{
    const int lane = lane_id();
    double* tmp = S.tmp + 24 * (a - 1);
    double ccs[4][3];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < 3; ++k) ccs[j][k] = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int col = 11 - i;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int k = 0; k < 3; ++k) ccs[j][k] += S.betas[a][i] * S.V12[(3 * j + k) * 12 + col];
    }
    auto pc = [&](int i, int j) {
        const double* al = alphas + 4 * i;
        return al[0] * ccs[0][j] + al[1] * ccs[1][j] + al[2] * ccs[2][j] + al[3] * ccs[3][j];
    };
    if (pc(0, 2) < 0.0) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int k = 0; k < 3; ++k) ccs[j][k] = -ccs[j][k];
    }
    wave_det_sum<3>(n, [&](int i, double* c) { c[0] = pc(i, 0); c[1] = pc(i, 1); c[2] = pc(i, 2); }, tmp);
    wave_lds_sync();
    double pc0[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) pc0[j] = tmp[j] / n;
    wave_lds_sync();
    wave_det_sum<9>(n, [&](int i, double* c) {
        double p[3] = {pc(i, 0), pc(i, 1), pc(i, 2)};
        for (int j = 0; j < 3; ++j)
            for (int k = 0; k < 3; ++k) c[j * 3 + k] = (p[j] - pc0[j]) * (pws[3 * i + k] - S.pw0[k]);
    }, tmp);
    wave_lds_sync();
    if (lane == 0) {
        double abt[9], w[3], V[9];
        for (int q = 0; q < 9; ++q) abt[q] = tmp[q];
        svd_jacobi<3, 3>(abt, w, V);
        double* R = S.Rs[a];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                R[i * 3 + j] = abt[i * 3 + 0] * V[j * 3 + 0] + abt[i * 3 + 1] * V[j * 3 + 1] + abt[i * 3 + 2] * V[j * 3 + 2];
        if (det3(R) < 0) { R[6] = -R[6]; R[7] = -R[7]; R[8] = -R[8]; }
        for (int i = 0; i < 3; ++i)
            S.ts[a][i] = pc0[i] - (R[i * 3] * S.pw0[0] + R[i * 3 + 1] * S.pw0[1] + R[i * 3 + 2] * S.pw0[2]);
    }
    wave_lds_sync();
    {
        const double* R = S.Rs[a];
        const double* t = S.ts[a];
        const double fu = K[0], fv = K[4], uc = K[2], vc = K[5];
        wave_det_sum<1>(n, [&](int i, double* c) {
            const double* pw = pws + 3 * i;
            double Xc = R[0] * pw[0] + R[1] * pw[1] + R[2] * pw[2] + t[0];
            double Yc = R[3] * pw[0] + R[4] * pw[1] + R[5] * pw[2] + t[1];
            double inv_Zc = 1.0 / (R[6] * pw[0] + R[7] * pw[1] + R[8] * pw[2] + t[2]);
            double ue = uc + fu * Xc * inv_Zc;
            double ve = vc + fv * Yc * inv_Zc;
            double u = us[2 * i], v = us[2 * i + 1];
            c[0] = sqrt((u - ue) * (u - ue) + (v - ve) * (v - ve));
        }, tmp);
    }
    wave_lds_sync();
    if (lane == 0) S.rep[a] = tmp[0] / n;
}

// EPnP (epnp::compute_pose), all threads of the block; n >= 4
VO_DEV void epnp_block(EpnpShared& S, const double* K, const double* pws, const double* us, double* alphas,
                       double* pcs, int n, double* Rout, double* tout)
{
    const int tid = threadIdx.x;
    if (wave_id() == 0)
        wave_det_sum<3>(n, [&](int i, double* c) { c[0] = pws[3 * i]; c[1] = pws[3 * i + 1]; c[2] = pws[3 * i + 2]; }, S.tmp);
    __syncthreads();
    if (tid == 0) for (int j = 0; j < 3; ++j) S.pw0[j] = S.cws[0][j] = S.tmp[j] / n;
    __syncthreads();
    if (wave_id() == 0)
        wave_det_sum<9>(n, [&](int i, double* c) {
            double d[3];
            for (int j = 0; j < 3; ++j) d[j] = pws[3 * i + j] - S.cws[0][j];
            for (int a = 0; a < 3; ++a) for (int b = 0; b < 3; ++b) c[a * 3 + b] = d[a] * d[b];
        }, S.tmp);
    __syncthreads();
    if (tid == 0) {
        double cov[9], dc[3], Vc[9];
        for (int q = 0; q < 9; ++q) cov[q] = S.tmp[q];
        svd_jacobi<3, 3>(cov, dc, Vc);
        for (int i = 1; i < 4; ++i) {
            double k = sqrt(dc[i - 1] / n);
            for (int j = 0; j < 3; ++j) S.cws[i][j] = S.cws[0][j] + k * cov[j * 3 + (i - 1)];
        }
        double CC[9], w[3], V[9];
        for (int i = 0; i < 3; ++i)
            for (int j = 1; j < 4; ++j) CC[3 * i + j - 1] = S.cws[j][i] - S.cws[0][i];
        svd_jacobi<3, 3>(CC, w, V);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                double s = 0;
                for (int k = 0; k < 3; ++k) if (w[k] > DBL_EPSILON * w[0] * 3) s += V[i * 3 + k] * CC[j * 3 + k] / w[k];
                S.CCi[i * 3 + j] = s;
            }
    }
    __syncthreads();
    for (int i = tid; i < n; i += blockDim.x) {
        const double* pi = pws + 3 * i;
        double* a = alphas + 4 * i;
        for (int j = 0; j < 3; ++j)
            a[1 + j] = S.CCi[3 * j] * (pi[0] - S.cws[0][0]) + S.CCi[3 * j + 1] * (pi[1] - S.cws[0][1]) +
                       S.CCi[3 * j + 2] * (pi[2] - S.cws[0][2]);
        a[0] = 1.0 - a[1] - a[2] - a[3];
    }
    __syncthreads();
    PNPPROF(10);
    // M^T M upper triangle (78 entries): one pass over the points, 4 waves x ~20 entries
    const double fu = K[0], fv = K[4], uc = K[2], vc = K[5];
    __shared__ double up[78];
    switch (wave_id()) {
        case 0: epnp_mtm_part<0, 20>(n, alphas, us, fu, fv, uc, vc, up); break;
        case 1: epnp_mtm_part<20, 40>(n, alphas, us, fu, fv, uc, vc, up); break;
        case 2: epnp_mtm_part<40, 60>(n, alphas, us, fu, fv, uc, vc, up); break;
        default: epnp_mtm_part<60, 78>(n, alphas, us, fu, fv, uc, vc, up); break;
    }
    __syncthreads();
    PNPPROF(16);
    // 12x12 round-robin Jacobi SVD of M^T M by wave 0 in LDS (oracle: svd_jacobi_rr)
    if (wave_id() == 0) {
        for (int q = lane_id(); q < 144; q += 64) {
            int a = q / 12, bb = q - a * 12;
            if (a > bb) { const int t = a; a = bb; bb = t; }
            S.MtM[q] = up[a * 12 - a * (a - 1) / 2 + (bb - a)];
        }
        wave_lds_sync();
        svd_jacobi_wave_rr<12, 12>(S.MtM, S.dM, S.V12, S.tmp);
    }
    __syncthreads();
    PNPPROF(11);
    if (tid == 0) {
        epnp_L6x10(S.V12, S.L);
        for (int j = 0; j < 6; ++j) {
            const double* p = S.cws[PAIR_A[j]];
            const double* r = S.cws[PAIR_B[j]];
            S.rho[j] = (p[0] - r[0]) * (p[0] - r[0]) + (p[1] - r[1]) * (p[1] - r[1]) + (p[2] - r[2]) * (p[2] - r[2]);
        }
    }
    __syncthreads();
    // the three beta approximations are independent: lane 0 of waves 0..2 computes one each,
    // and its wave goes straight on to that approximation's compute_R_and_t (no block barrier
    // between them, so the two shorter chains' R, t hide under the longest one's betas).  The
    // oracle runs approximation 1's R,t before computing approximation 2's betas; the betas do
    // not depend on R,t, so the order between approximations is immaterial.  compute_R_and_t's
    // world centroid pw0 is the same sum of the same points in the same order as the first
    // control point cws[0] (set with it above), so it is not summed again.
    const int wv = wave_id();
    if (wv < 3) {
        if (lane_id() == 0) {
            if (wv == 0) {
                double A[24], b4[4];
                const int cols[4] = {0, 1, 3, 6};
                for (int i = 0; i < 6; ++i) for (int j = 0; j < 4; ++j) A[i * 4 + j] = S.L[i * 10 + cols[j]];
                lsq_svd<6, 4>(A, S.rho, b4);
                PNPPROF_T(17, 0);
                double* B = S.betas[1];
                if (b4[0] < 0) { B[0] = sqrt(-b4[0]); B[1] = -b4[1] / B[0]; B[2] = -b4[2] / B[0]; B[3] = -b4[3] / B[0]; }
                else { B[0] = sqrt(b4[0]); B[1] = b4[1] / B[0]; B[2] = b4[2] / B[0]; B[3] = b4[3] / B[0]; }
                epnp_gauss_newton(S.L, S.rho, B);
                PNPPROF_T(18, 0);
            } else if (wv == 1) {
                double A[18], b3[3];
                for (int i = 0; i < 6; ++i) for (int j = 0; j < 3; ++j) A[i * 3 + j] = S.L[i * 10 + j];
                lsq_svd<6, 3>(A, S.rho, b3);
                PNPPROF_T(24, 64);
                double* B = S.betas[2];
                if (b3[0] < 0) { B[0] = sqrt(-b3[0]); B[1] = (b3[2] < 0) ? sqrt(-b3[2]) : 0.0; }
                else { B[0] = sqrt(b3[0]); B[1] = (b3[2] > 0) ? sqrt(b3[2]) : 0.0; }
                if (b3[1] < 0) B[0] = -B[0];
                B[2] = 0.0; B[3] = 0.0;
                epnp_gauss_newton(S.L, S.rho, B);
                PNPPROF_T(25, 64);
            } else {
                double A[30], b5[5];
                for (int i = 0; i < 6; ++i) for (int j = 0; j < 5; ++j) A[i * 5 + j] = S.L[i * 10 + j];
                lsq_svd<6, 5>(A, S.rho, b5);
                PNPPROF_T(19, 128);
                double* B = S.betas[3];
                if (b5[0] < 0) { B[0] = sqrt(-b5[0]); B[1] = (b5[2] < 0) ? sqrt(-b5[2]) : 0.0; }
                else { B[0] = sqrt(b5[0]); B[1] = (b5[2] > 0) ? sqrt(b5[2]) : 0.0; }
                if (b5[1] < 0) B[0] = -B[0];
                B[2] = b5[3] / B[0]; B[3] = 0.0;
                epnp_gauss_newton(S.L, S.rho, B);
                PNPPROF_T(23, 128);
            }
        }
        wave_lds_sync();
        epnp_R_and_t_wave(S, wv + 1, K, pws, us, alphas, n);
    }
    __syncthreads();
    PNPPROF(13);
    if (tid == 0) {
        int N = 1;
        if (S.rep[2] < S.rep[1]) N = 2;
        if (S.rep[3] < S.rep[N]) N = 3;
        for (int q = 0; q < 9; ++q) Rout[q] = S.Rs[N][q];
        for (int q = 0; q < 3; ++q) tout[q] = S.ts[N][q];
    }
    __syncthreads();
}

// ------------------------------------------------------------------ PnP-RANSAC
#define HYP 64
#ifndef VO_PNP_CH1
#define VO_PNP_CH1 32
#endif

struct PnPArgs {
    double K[9];
    float thr;              // (float)(reprojectionError^2)
    double conf;
    int iters;
    int min_points;
    const float* obj;       // [B][cap][3]
    const float* img;       // [B][cap][2]
    const int32_t* counts;
    int cap;
    const int32_t* chain_status;
    double* work;           // [B][work_stride]
    int64_t work_stride;
    int32_t* iwork;         // [B][iwork_stride]
    int64_t iwork_stride;
    // outputs (may alias iwork/work for the engine)
    double* rvec;           // [B][3]
    double* tvec;           // [B][3]
    int32_t* success;       // [B]
    uint8_t* mask;          // [B][cap]
    int32_t* n_inl;         // [B]
};

// getSubset for CH hypotheses (oracle get_subset: four draws rng % n per hypothesis, a draw equal
// to an earlier one of the same hypothesis drawn again), by one whole wave.  Lane 0 runs the
// generator -- one multiply-add per value, no division -- for the 4 CH values a round without
// repeats consumes, storing each value and the state after it; the lanes reduce them mod n in
// parallel and check each hypothesis's four for a repeat.  The hypotheses before the first one
// with a repeat take their four values as drawn; from that one on, lane 0 applies the serial rule
// to the stored values (drawing past them if it needs more): the same draws in the same order.
// rng (lane 0's copy) ends past the last value used.
VO_DEV void pnp_subsets(int CH, uint32_t un, uint64_t& rng, int (*sub)[4], uint32_t* res, uint64_t* st)
{
    const int lane = lane_id(), R = 4 * CH;
    if (lane == 0) {
        uint64_t g = rng;
        for (int i = 0; i < R; ++i) {
            g = (uint64_t)(uint32_t)g * 4164903690ULL + (g >> 32);       // rng_next
            res[i] = (uint32_t)g;
            st[i] = g;
        }
    }
    wave_lds_sync();
    for (int i = lane; i < R; i += 64) res[i] = res[i] % un;
    wave_lds_sync();
    int bad = CH;
    for (int h0 = 0; h0 < CH; h0 += 64) {
        const int h = h0 + lane;
        bool rep = false;
        if (h < CH) {
            const uint32_t a = res[4 * h], b = res[4 * h + 1], c = res[4 * h + 2], d = res[4 * h + 3];
            rep = b == a || c == a || c == b || d == a || d == b || d == c;
        }
        const unsigned long long m = __ballot(rep);
        if (m) { bad = h0 + __ffsll((long long)m) - 1; break; }
    }
    for (int h = lane; h < bad; h += 64) {
        sub[h][0] = (int)res[4 * h]; sub[h][1] = (int)res[4 * h + 1];
        sub[h][2] = (int)res[4 * h + 2]; sub[h][3] = (int)res[4 * h + 3];
    }
    if (lane == 0) {
        int p = 4 * bad;
        uint64_t g = p > 0 ? st[p - 1] : rng;
        auto draw = [&]() -> int {
            int v;
            if (p < R) { v = (int)res[p]; g = st[p]; }
            else v = (int)(rng_next(g) % un);
            ++p;
            return v;
        };
        for (int h = bad; h < CH; ++h) {
            const int s0 = draw();
            int s1, s2, s3;
            do { s1 = draw(); } while (s1 == s0);
            do { s2 = draw(); } while (s2 == s0 || s2 == s1);
            do { s3 = draw(); } while (s3 == s0 || s3 == s1 || s3 == s2);
            sub[h][0] = s0; sub[h][1] = s1; sub[h][2] = s2; sub[h][3] = s3;
        }
        rng = g;
    }
}

// defer (k_pnp_tri): on the refit path, leave the final pose in defer[0..12) (R row-major, t)
// with *pend = 1 instead of forming rvec here, so that the epilogue's Rodrigues pair runs beside
// its landmark compaction (pnp_apply_split); *pend stays as the caller set it (0) otherwise
VO_DEV void pnp_ransac_block(const PnPArgs& A, double* defer = nullptr, int* pend = nullptr)
{
    __shared__ int sub[HYP][4];
    __shared__ double mdl[HYP][12];
    __shared__ int valid[HYP], cnt[HYP];
    __shared__ double bestm[12];
    __shared__ int sh[8];
    __shared__ int lds16[16];
    __shared__ EpnpShared S;
    __shared__ uint32_t sub_res[4 * HYP];
    __shared__ uint64_t sub_st[4 * HYP];
    __shared__ double den_ld[HYP];
    __shared__ int den_ok[HYP];
    __shared__ double lnum_sh;
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    if (A.chain_status && A.chain_status[b] != 0) return;
    const int n = A.counts[b];
    const float* obj = A.obj + (int64_t)b * A.cap * 3;
    const float* img = A.img + (int64_t)b * A.cap * 2;
    uint8_t* mask = A.mask + (int64_t)b * A.cap;
    if (n < 4 || n < A.min_points) {
        if (tid == 0) { A.success[b] = 0; A.n_inl[b] = 0; }
        return;
    }
    const CamK k = camk(A.K);
    if (n == 4) {
        if (tid == 0) {
            double o[12], im[8], R[9], t[3];
            for (int i = 0; i < 12; ++i) o[i] = obj[i];
            for (int i = 0; i < 8; ++i) im[i] = img[i];
            int ok = p3p_solve4(k, o, im, R, t);
            A.success[b] = ok;
            A.n_inl[b] = ok ? 4 : 0;
            if (ok) {
                rodrigues_m2v(R, A.rvec + 3 * b);
                for (int q = 0; q < 3; ++q) A.tvec[3 * b + q] = t[q];
            }
            for (int i = 0; i < 4; ++i) mask[i] = ok ? 1 : 0;
        }
        return;
    }
    PNPPROF(0);
    uint64_t rng = ~0ULL;   // only thread 0's copy is used
    if (tid == 0) { sh[0] = 0; sh[1] = A.iters > 1 ? A.iters : 1; sh[2] = 0; }
    __syncthreads();
    while (true) {
        const int it0 = sh[0];
        const int niters0 = sh[1];
        if (it0 >= niters0) break;
        // a smaller first round: with the usual inlier ratios the adaptive iteration count
        // drops below it there, and fewer diverging P3P lanes and inlier counts finish sooner
        const int CH = it0 == 0 ? VO_PNP_CH1 : HYP;
        PNPPROF(1);
        if (wave_id() == 0) pnp_subsets(CH, (uint32_t)n, rng, sub, sub_res, sub_st);
        else if (it0 == 0 && tid == 64) lnum_sh = ransac_log_num(A.conf);    // log(1 - confidence), once
        __syncthreads();
        PNPPROF(6);
        {
            // four lanes per hypothesis, one P3P solution each (p3p_solution); the lanes then
            // apply p3p_solve4's rule (first solution with a strictly smaller 4th-point error).
            // The hypotheses are spread over all waves (CH / waves each): a wave's P3P time is
            // that of its slowest root bracketing / eigen-sweep count, so fewer per wave finish sooner.
            const int lane = lane_id(), hpw = CH / (blockDim.x >> 6), hq = lane >> 2, sol = lane & 3;
            const int h = hq < hpw ? wave_id() * hpw + hq : CH;
            double R[9], t[3], e = 0.0;
            int ok = 0;
            if (h < CH && it0 + h < niters0) {
                double o[12], im[8];
                for (int j = 0; j < 4; ++j) {
                    const int id = sub[h][j];
                    o[3 * j] = obj[3 * id]; o[3 * j + 1] = obj[3 * id + 1]; o[3 * j + 2] = obj[3 * id + 2];
                    im[2 * j] = img[2 * id]; im[2 * j + 1] = img[2 * id + 1];
                }
                ok = p3p_solution(k, o, im, sol, R, t, &e);
            }
            int bsol = -1;
            double be = 0.0;
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) {
                const int oks = __shfl(ok, (lane & ~3) | s2, 64);
                const double es = __shfl(e, (lane & ~3) | s2, 64);
                if (oks && (bsol < 0 || es < be)) { bsol = s2; be = es; }
            }
            if (h < CH) {
                if (sol == 0) valid[h] = bsol >= 0;
                if (sol == bsol) {
                    for (int q = 0; q < 9; ++q) mdl[h][q] = R[q];
                    for (int q = 0; q < 3; ++q) mdl[h][9 + q] = t[q];
                }
            }
        }
        __syncthreads();
        PNPPROF(2);
        {
            // scoring in the order the sequential rule below visits the hypotheses, one per wave
            // at a time: a hypothesis at or past the running adaptive iteration count is never
            // looked at, so the batches stop once it is reached (same result as scoring all CH)
            // Two hypotheses per wave per batch (h and h + nw), scored in one pass over the points
            // (each point loaded once, two independent error chains): with the usual adaptive
            // counts (2-8) the first batch already reaches the final count.
            const int w = wave_id(), lane = lane_id(), nw = blockDim.x >> 6, HB = 2 * nw;
            for (int h0 = 0; h0 < CH; h0 += HB) {
                const int nit = sh[1];
                if (it0 + h0 >= nit) break;                           // block-uniform
                const int ha = h0 + w, hb = h0 + w + nw;
                // a hypothesis at or past the running count is never looked at by the rule below
                const bool va = ha < CH && it0 + ha < nit && valid[ha];
                const bool vb = hb < CH && it0 + hb < nit && valid[hb];
                if (va || vb) {
                    const double* Ra = mdl[va ? ha : hb];
                    const double* Rb = mdl[vb ? hb : ha];
                    int ca = 0, cb = 0;
                    for (int i = lane; i < n; i += 64) {
                        const float X0 = obj[3 * i], X1 = obj[3 * i + 1], X2 = obj[3 * i + 2], u = img[2 * i], v = img[2 * i + 1];
                        if (va) ca += pnp_err(Ra, Ra + 9, k, X0, X1, X2, u, v) <= A.thr;
                        if (vb) cb += pnp_err(Rb, Rb + 9, k, X0, X1, X2, u, v) <= A.thr;
                    }
                    if (va) ca = wave_sum_i32(ca);
                    if (vb) cb = wave_sum_i32(cb);
                    if (lane == 0) {
                        if (va) cnt[ha] = ca;
                        if (vb) cnt[hb] = cb;
                    }
                }
                __syncthreads();
                if (h0 == 0) PNPPROF(28);
                if (w == 0) {
                    // the expensive half of every update this batch can make (its log), one lane
                    // per hypothesis; lane 0 then applies the sequential rule with them
                    const int h1 = h0 + HB < CH ? h0 + HB : CH;
                    const int hh = h0 + lane;
                    if (hh < h1 && it0 + hh < nit && valid[hh]) {
                        double ld = 0.0;
                        den_ok[hh] = ransac_niters_den((double)(n - cnt[hh]) / n, 4, &ld);
                        den_ld[hh] = ld;
                    }
                    wave_lds_sync();
                    if (lane == 0) {
                        int niters = sh[1], best = sh[2];
                        for (int q = h0; q < h1; ++q) {
                            if (it0 + q >= niters) break;
                            if (!valid[q]) continue;
                            const int good = cnt[q];
                            if (good > (best > 3 ? best : 3)) {
                                best = good;
                                for (int r = 0; r < 12; ++r) bestm[r] = mdl[q][r];
                                niters = ransac_niters_fin(lnum_sh, den_ok[q], den_ld[q], niters);
                            }
                        }
                        sh[1] = niters;
                        sh[2] = best;
                    }
                }
                __syncthreads();
                if (h0 == 0) PNPPROF(29);
            }
        }
        if (tid == 0) sh[0] = it0 + CH;
        __syncthreads();
    }
    PNPPROF(3);
    PNPVAL(20, sh[0]);
    PNPVAL(21, sh[1]);
    PNPVAL(22, sh[2]);
    if (sh[2] <= 0) {
        if (tid == 0) { A.success[b] = 0; A.n_inl[b] = 0; }
        for (int i = tid; i < n; i += blockDim.x) mask[i] = 0;
        return;
    }
    // inlier mask of the best model + ordered compaction into fp64 scratch
    double* work = A.work + (int64_t)b * A.work_stride;
    double* pws = work;                       // [n][3]
    double* us = work + 3 * A.cap;            // [n][2]
    double* alphas = work + 5 * A.cap;        // [n][4]
    double* pcs = work + 9 * A.cap;           // [n][3]
    int m = 0;
    for (int base = 0; base < n; base += blockDim.x) {
        const int i = base + tid;
        bool in = false;
        if (i < n) {
            in = pnp_err(bestm, bestm + 9, k, obj[3 * i], obj[3 * i + 1], obj[3 * i + 2], img[2 * i], img[2 * i + 1]) <= A.thr;
            mask[i] = in ? 1 : 0;
        }
        int tot;
        const int pos = m + block_scan_flag(in, lds16, &tot);
        if (in) {
            pws[3 * pos] = obj[3 * i]; pws[3 * pos + 1] = obj[3 * i + 1]; pws[3 * pos + 2] = obj[3 * i + 2];
            const double un = ((double)img[2 * i] - k.cx) * k.ifx, vn = ((double)img[2 * i + 1] - k.cy) * k.ify;
            us[2 * pos] = un * k.fx + k.cx;
            us[2 * pos + 1] = vn * k.fy + k.cy;
        }
        m += tot;
    }
    __syncthreads();
    __shared__ double Rfin[9], tfin[3];
    PNPPROF(4);
    epnp_block(S, A.K, pws, us, alphas, pcs, m, Rfin, tfin);
    PNPPROF(5);
    if (tid == 0) {
        if (defer) {
            for (int q = 0; q < 9; ++q) defer[q] = Rfin[q];
            for (int q = 0; q < 3; ++q) defer[9 + q] = tfin[q];
            *pend = 1;
        } else {
            rodrigues_m2v(Rfin, A.rvec + 3 * b);
        }
        for (int q = 0; q < 3; ++q) A.tvec[3 * b + q] = tfin[q];
        A.success[b] = 1;
        A.n_inl[b] = m;
    }
}

// engine epilogue of the PnP step (:342-358): guard, inlier filtering, Rodrigues, inversion
VO_DEV void pnp_apply_block(const vo_dims& d, const vo_state& s, const double* rvec, const double* tvec,
                            const int32_t* success, const uint8_t* mask_all)
{
    __shared__ int lds[16];
    __shared__ double Rwc[9];
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    if (s.status[b] != 0) return;
    const int n = s.nL[b];
    if (n < 8) { if (tid == 0) s.status[b] = VO_ST_NOT_ENOUGH_KP; return; }
    if (!success[b]) { if (tid == 0) s.status[b] = VO_ST_PNP_FAILED; return; }
    const uint8_t* mask = mask_all + (int64_t)b * d.ncap;
    float* X = s.lm_X + (int64_t)b * d.ncap * 3;
    float* kp = s.lm_kp + (int64_t)b * d.ncap * 2;
    const int kcap = d.ncap > d.pcap ? d.ncap : d.pcap;
    float* outl = s.outl_kp + (int64_t)b * kcap * 2;
    float* inl = s.inl_kp + (int64_t)b * kcap * 2;
    int nin = 0, nout = 0;
    for (int base = 0; base < n; base += blockDim.x) {
        const int i = base + tid;
        const bool valid = i < n;
        const bool in = valid && mask[i];
        float x0 = 0, x1 = 0, x2 = 0, k0 = 0, k1 = 0;
        if (valid) { x0 = X[3 * i]; x1 = X[3 * i + 1]; x2 = X[3 * i + 2]; k0 = kp[2 * i]; k1 = kp[2 * i + 1]; }
        int tin;
        const int pre = block_scan_flag(in, lds, &tin);                 // every thread before tid is valid
        const int pin = nin + pre, pout = nout + (tid - pre);
        const int tout = (n - base < (int)blockDim.x ? n - base : (int)blockDim.x) - tin;
        if (in) {
            X[3 * pin] = x0; X[3 * pin + 1] = x1; X[3 * pin + 2] = x2;
            kp[2 * pin] = k0; kp[2 * pin + 1] = k1;
            inl[2 * pin] = k0; inl[2 * pin + 1] = k1;
        } else if (valid) {
            outl[2 * pout] = k0; outl[2 * pout + 1] = k1;
        }
        nin += tin;
        nout += tout;
        __syncthreads();
    }
    if (tid == 0) {
        s.nL[b] = nin;
        s.nInl[b] = nin;
        s.nOutl[b] = nout;
        rodrigues_v2m(rvec + 3 * b, Rwc);
        const int f = s.nF[b];
        if (f >= d.fcap) { s.status[b] = VO_ST_CAPACITY; return; }
        double* Rcw = s.pose_R + ((int64_t)b * d.fcap + f) * 9;
        double* tcw = s.pose_t + ((int64_t)b * d.fcap + f) * 3;
        const double* t = tvec + 3 * b;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) Rcw[i * 3 + j] = Rwc[j * 3 + i];
        // invert_transform :74-75, tnew = -Rnew @ t with Rnew = R.T: numpy hands the (column-
        // major) matrix to BLAS gemv, which accumulates the columns j = 0, 1, 2 with fused
        // multiply-adds -- reproduced here so the pose is bit-identical (tools/blas_order_probe.py)
        for (int i = 0; i < 3; ++i)
            tcw[i] = __builtin_fma(-Rcw[i * 3 + 2], t[2], __builtin_fma(-Rcw[i * 3 + 1], t[1], -Rcw[i * 3] * t[0]));
    }
}

// pnp_apply_block for k_pnp_tri, after pnp_ransac_block(A, defer, pend): lane 0 of wave 0 forms
// rvec from the deferred pose (Rodrigues, as pnp_ransac_block does), converts it back and writes
// the inverted pose, while wave 1 compacts the landmarks on its own (a wave-level scan over four
// 64-point chunks per pass, no block barrier): the same values in the same slots as
// pnp_apply_block, the two serial parts side by side
VO_DEV void pnp_apply_split(const vo_dims& d, const vo_state& s, double* rvec, const double* tvec,
                            const int32_t* success, const uint8_t* mask_all, const double* defer, int pend)
{
    const int b = blockIdx.x;
    const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
    // every wave reads the status before wave 0 may store VO_ST_CAPACITY below (a
    // wave reading it late skipped the landmark compaction); the block is whole here
    const int st0 = s.status[b], n = s.nL[b], ok = success[b];
    __syncthreads();
    if (st0 != 0) return;
    if (n < 8) { if (tid == 0) s.status[b] = VO_ST_NOT_ENOUGH_KP; return; }
    if (!ok) { if (tid == 0) s.status[b] = VO_ST_PNP_FAILED; return; }
    if (w == 0) {
        if (lane == 0) {
            double rv[3], Rwc[9];
            if (pend) {
                rodrigues_m2v(defer, rv);
                for (int q = 0; q < 3; ++q) rvec[3 * b + q] = rv[q];
            } else {
                for (int q = 0; q < 3; ++q) rv[q] = rvec[3 * b + q];
            }
            rodrigues_v2m(rv, Rwc);
            const int f = s.nF[b];
            if (f >= d.fcap) {
                s.status[b] = VO_ST_CAPACITY;
            } else {
                double* Rcw = s.pose_R + ((int64_t)b * d.fcap + f) * 9;
                double* tcw = s.pose_t + ((int64_t)b * d.fcap + f) * 3;
                const double* t = tvec + 3 * b;
                for (int i = 0; i < 3; ++i)
                    for (int j = 0; j < 3; ++j) Rcw[i * 3 + j] = Rwc[j * 3 + i];
                // invert_transform :74-75 in BLAS gemv's fused order (pnp_apply_block)
                for (int i = 0; i < 3; ++i)
                    tcw[i] = __builtin_fma(-Rcw[i * 3 + 2], t[2], __builtin_fma(-Rcw[i * 3 + 1], t[1], -Rcw[i * 3] * t[0]));
            }
        }
    } else if (w == 1) {
        const uint8_t* mask = mask_all + (int64_t)b * d.ncap;
        float* X = s.lm_X + (int64_t)b * d.ncap * 3;
        float* kp = s.lm_kp + (int64_t)b * d.ncap * 2;
        const int kcap = d.ncap > d.pcap ? d.ncap : d.pcap;
        float* outl = s.outl_kp + (int64_t)b * kcap * 2;
        float* inl = s.inl_kp + (int64_t)b * kcap * 2;
        const unsigned long long below = (1ull << lane) - 1ull;
        int nin = 0, nout = 0;
        for (int base = 0; base < n; base += 256) {
            // loads of the four chunks first (every write of this pass lands below base + 256 and
            // at or below its own source index, so no later read sees a moved point)
            float x0[4], x1[4], x2[4], k0[4], k1[4];
            bool in[4], valid[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int i = base + 64 * c + lane;
                valid[c] = i < n;
                in[c] = valid[c] && mask[i];
                x0[c] = x1[c] = x2[c] = k0[c] = k1[c] = 0.f;
                if (valid[c]) { x0[c] = X[3 * i]; x1[c] = X[3 * i + 1]; x2[c] = X[3 * i + 2]; k0[c] = kp[2 * i]; k1[c] = kp[2 * i + 1]; }
            }
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const unsigned long long mi = __ballot(in[c]), mv = __ballot(valid[c]);
                const int pre = __popcll(mi & below), tin = __popcll(mi), tv = __popcll(mv);
                const int pin = nin + pre, pout = nout + (lane - pre);      // valid lanes are a prefix
                if (in[c]) {
                    X[3 * pin] = x0[c]; X[3 * pin + 1] = x1[c]; X[3 * pin + 2] = x2[c];
                    kp[2 * pin] = k0[c]; kp[2 * pin + 1] = k1[c];
                    inl[2 * pin] = k0[c]; inl[2 * pin + 1] = k1[c];
                } else if (valid[c]) {
                    outl[2 * pout] = k0[c]; outl[2 * pout + 1] = k1[c];
                }
                nin += tin;
                nout += tv - tin;
            }
        }
        if (lane == 0) {
            s.nL[b] = nin;
            s.nInl[b] = nin;
            s.nOutl[b] = nout;
        }
    }
}

__global__ void __launch_bounds__(256) k_pnp_ransac(PnPArgs A) { pnp_ransac_block(A); }

__global__ void __launch_bounds__(256) k_pnp_apply(vo_dims d, vo_state s, const double* rvec, const double* tvec,
                                                   const int32_t* success, const uint8_t* mask_all)
{
    pnp_apply_block(d, s, rvec, tvec, success, mask_all);
}

// the engine's PnP stage as one launch: RANSAC + EPnP, then (after a block barrier, which
// makes thread 0's rvec / tvec / success visible to the block) the epilogue -- a second,
// separate launch had to wait for CUs behind the other stream group's LK blocks
// At most 256 registers per lane (VGPR + AGPR) -- two waves per SIMD, some spilled to scratch --
// so that two chains' blocks fit on one CU: with 384 chains per launch on 256 CUs, a block
// needing a whole CU left a third of the chains to start only after the other stream group's LK
// flood (which refills every freed wave slot) had drained.
#ifndef VO_PNP_WPE
#define VO_PNP_WPE 2
#endif
template <int WPE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, 8)))
k_pnp_fused(PnPArgs A, vo_dims d, vo_state s)
{
    pnp_ransac_block(A);
    __syncthreads();
    pnp_apply_block(d, s, A.rvec, A.tvec, A.success, A.mask);
}

// ------------------------------------------------------------------ triangulation
// The reference forms its projection matrices and camera-frame depths with numpy
// matmuls (VisualOdometryPipeLine.py:74-75 invert_transform, :157-168, :170-171), which
// OpenBLAS evaluates as fused multiply-add chains whose order depends on the operands'
// memory layout (tools/blas_order_probe.py checks the models below on the host):
//   C-order matrix @ vector  (gemv, dot products)   fma(a2,b2, fma(a0,b0, a1*b1))
//   F-order matrix @ vector  (gemv, column axpys)   fma(a2,b2, fma(a1,b1, a0*b0))
//   K @ [R | t]              (gemm)                 fma(a2,b2, fma(a1,b1, a0*b0))
// Every 3x3 gemm of check_baseline ((R_cur^T R_past)^T, then @ K_inv) is the k-order chain.
// R_WC = R_CW.T is F-order for the identity pose 0 and the bootstrap pose 1 (recoverPose
// returns a C-order R) and C-order for every later pose (R_CW = Rodrigues(rvec).T).  The
// triangulated point depends on every bit of the two projection matrices, so they are
// reproduced exactly; a landmark coordinate near 0 otherwise differs in its last float bit
// (found 619 frames into the C2 chain, tools/diag_long.py).
VO_DEV double dot_c012(const double* a, const double* b)
{
    return __builtin_fma(a[2], b[2], __builtin_fma(a[1], b[1], a[0] * b[0]));
}
VO_DEV double dot_c102(const double* a, const double* b)
{
    return __builtin_fma(a[2], b[2], __builtin_fma(a[0], b[0], a[1] * b[1]));
}
// (R_WC, t_WC) = invert_transform(R_CW, t_CW) of pose p: R_WC = R_CW^T, t_WC = (-R_WC) @ t_CW
VO_DEV void pose_inverse(const double* Rcw, const double* tcw, int p, double* Rwc, double* twc)
{
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) Rwc[i * 3 + j] = Rcw[j * 3 + i];
    for (int i = 0; i < 3; ++i) {
        const double a[3] = {-Rwc[i * 3], -Rwc[i * 3 + 1], -Rwc[i * 3 + 2]};
        twc[i] = p >= 2 ? dot_c102(a, tcw) : dot_c012(a, tcw);
    }
}
// P = K @ np.hstack((R_WC, t_WC)), 3x4
VO_DEV void proj_matrix(const double* K, const double* Rwc, const double* twc, double* P)
{
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 4; ++j) {
            const double m[3] = {j < 3 ? Rwc[j] : twc[0], j < 3 ? Rwc[3 + j] : twc[1], j < 3 ? Rwc[6 + j] : twc[2]};
            P[i * 4 + j] = dot_c012(K + i * 3, m);
        }
}
// z of (R_WC @ X + t_WC) (:157-168; X float32 promoted to float64)
VO_DEV double depth_of(const double* Rwc, const double* twc, int p, const float* X)
{
    const double x[3] = {(double)X[0], (double)X[1], (double)X[2]};
    return (p >= 2 ? dot_c102(Rwc + 6, x) : dot_c012(Rwc + 6, x)) + twc[2];
}

struct TriArgs {
    vo_dims d;
    vo_state s;
    double K[9], Kinv[9];
    double min_d, max_d;
    double cos_thr;        // retain iff clip(cos) >= cos_thr  <=>  degrees(arccos(cos)) < min_baseline_angle
    int min_frames;
    int force;
    int compact;           // k_pnp_tri: run feature_tracking's filtering first (vo_filter_pnp_triangulate)
};

// Shared per-chain context of the triangulation passes: the current pose (R_CW, t_CW), its
// inverse and projection matrix, computed by thread 0.
struct TriShared {
    double Rc[9], tc[3], Rcwc[9], tcwc[3], Pc[12];
    int fail, m;
};

// false: the chain does not triangulate this step (status set, or :366's nC <= 1)
VO_DEV bool tri_setup(const TriArgs& A, TriShared& sh)
{
    const int b = blockIdx.x;
    const vo_dims& d = A.d;
    const vo_state& s = A.s;
    if (s.status[b] != 0) return false;
    if (!A.force && s.nC[b] <= 1) return false;                       // :366
    if (threadIdx.x == 0) {
        const int nF = s.nF[b];
        const double* poseR = s.pose_R + (int64_t)b * d.fcap * 9;
        const double* poset = s.pose_t + (int64_t)b * d.fcap * 3;
        sh.fail = 0;
        sh.m = 0;
        // current pose (R_CW, t_CW) is slot nF; (R_WC, t_WC) = (R^T, -R^T t)
        for (int i = 0; i < 9; ++i) sh.Rc[i] = poseR[(int64_t)nF * 9 + i];
        for (int i = 0; i < 3; ++i) sh.tc[i] = poset[(int64_t)nF * 3 + i];
        pose_inverse(sh.Rc, sh.tc, nF, sh.Rcwc, sh.tcwc);
        proj_matrix(A.K, sh.Rcwc, sh.tcwc, sh.Pc);
    }
    __syncthreads();
    return true;
}

// Three passes over the candidates (results identical to one pass, the reference's loop
// :171-206): (1) the frame gate and check_baseline, listing the candidates that reach
// cv2.triangulatePoints; (2) the triangulations, one listed candidate per thread -- the 4x4
// Jacobi SVD is a long serial FP64 chain, so a chunk of 256 candidates with a few of them
// triangulating cost as much as a chunk of 256 triangulations; (3) the ordered append /
// compaction.  Scratch: the list, flags and list length in iwork, the points in work (PnP is
// done with it).  The engine's step runs the three in the PnP block (k_pnp_tri); vo_triangulate
// runs pass 2 over several blocks per chain (k_tri_solve).
VO_DEV void tri_gate(const TriArgs& A, TriShared& sh)
{
    const int b = blockIdx.x, tid = threadIdx.x;
    const vo_dims& d = A.d;
    const vo_state& s = A.s;
    const int nC = s.nC[b], nF = s.nF[b];
    const double* poseR = s.pose_R + (int64_t)b * d.fcap * 9;
    const float* ck = s.c_kp + (int64_t)b * d.pcap * 2;
    const float* cf = s.c_first + (int64_t)b * d.pcap * 2;
    const int32_t* ct = s.c_tau + (int64_t)b * d.pcap;
    const int kmax = d.ncap > d.pcap ? d.ncap : d.pcap;
    int32_t* tlist = s.iwork + (int64_t)b * d.iwork_stride;          // [m] candidate indices
    int32_t* tacc = tlist + kmax;                                      // [nC] 1 = becomes a landmark
    const double* Rc = sh.Rc;
    for (int i = tid; i < nC; i += blockDim.x) {
        const float k0 = ck[2 * i], k1 = ck[2 * i + 1], f0 = cf[2 * i], f1 = cf[2 * i + 1];
        const int tau = ct[i];
        bool tri = false;
        if (!(nF > 1 && nF - tau <= A.min_frames)) {                    // else retained, :175-178
            const double* Rp = poseR + (int64_t)tau * 9;
            // check_baseline :117-147: v_cur = K^-1 [u;1], v_past = ((R_cur^T R_past)^T K^-1) [u_f;1]
            double vc[3], vp[3], rel[9], Mr[9];
            const double uc[3] = {(double)k0, (double)k1, 1.0};
            for (int r = 0; r < 3; ++r) vc[r] = dot_c102(A.Kinv + r * 3, uc);      // K_inv (C-order) @ v
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c)
                    rel[c * 3 + r] = __builtin_fma(Rc[6 + r], Rp[6 + c], __builtin_fma(Rc[3 + r], Rp[3 + c], Rc[r] * Rp[c]));
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c)
                    Mr[r * 3 + c] = __builtin_fma(rel[r * 3 + 2], A.Kinv[6 + c],
                                                  __builtin_fma(rel[r * 3 + 1], A.Kinv[3 + c], rel[r * 3] * A.Kinv[c]));
            const double uf[3] = {(double)f0, (double)f1, 1.0};
            for (int r = 0; r < 3; ++r) vp[r] = dot_c102(Mr + r * 3, uf);            // matmul output (C-order) @ v
            double dot = vc[0] * vp[0] + vc[1] * vp[1] + vc[2] * vp[2];
            double nc = sqrt(vc[0] * vc[0] + vc[1] * vc[1] + vc[2] * vc[2]);
            double np = sqrt(vp[0] * vp[0] + vp[1] * vp[1] + vp[2] * vp[2]);
            double cs = dot / (nc * np);
            cs = cs < -1.0 ? -1.0 : (cs > 1.0 ? 1.0 : cs);
            // np.degrees(np.arccos(c)) < min_baseline_angle (:144-147) without a device acos:
            // arccos is monotone, so the gate is c >= the smallest double the host's own
            // np.arccos puts inside the angle (engine.baseline_cos_threshold); NaN stays false
            tri = !(cs >= A.cos_thr);                                   // else retained
        }
        tacc[i] = 0;
        if (tri) tlist[atomicAdd(&sh.m, 1)] = i;
    }
    __syncthreads();
}

// pass 2 over list entries j0, j0 + stride, ... (m entries)
VO_DEV void tri_solve(const TriArgs& A, const TriShared& sh, int m, int j0, int stride)
{
    const int b = blockIdx.x;
    const vo_dims& d = A.d;
    const vo_state& s = A.s;
    const int nF = s.nF[b];
    const double* poseR = s.pose_R + (int64_t)b * d.fcap * 9;
    const double* poset = s.pose_t + (int64_t)b * d.fcap * 3;
    const float* ck = s.c_kp + (int64_t)b * d.pcap * 2;
    const float* cf = s.c_first + (int64_t)b * d.pcap * 2;
    const int32_t* ct = s.c_tau + (int64_t)b * d.pcap;
    const int kmax = d.ncap > d.pcap ? d.ncap : d.pcap;
    const int32_t* tlist = s.iwork + (int64_t)b * d.iwork_stride;
    int32_t* tacc = s.iwork + (int64_t)b * d.iwork_stride + kmax;
    float* tX = (float*)(s.work + (int64_t)b * d.work_stride);          // [nC][3] its point
    for (int j = j0; j < m; j += stride) {
        const int i = tlist[j];
        const float k0 = ck[2 * i], k1 = ck[2 * i + 1], f0 = cf[2 * i], f1 = cf[2 * i + 1];
        const int tau = ct[i];
        const double* Rp = poseR + (int64_t)tau * 9;
        const double* tp = poset + (int64_t)tau * 3;
        double Rpw[9], tpw[3], Pp[12];
        pose_inverse(Rp, tp, tau, Rpw, tpw);
        proj_matrix(A.K, Rpw, tpw, Pp);
        double X4[4];
        tri_one(Pp, sh.Pc, (double)f0, (double)f1, (double)k0, (double)k1, X4);
        const float w4 = (float)X4[3];
        float Xo[3];
        Xo[0] = (float)X4[0] / w4;
        Xo[1] = (float)X4[1] / w4;
        Xo[2] = (float)X4[2] / w4;
        const double zc = depth_of(sh.Rcwc, sh.tcwc, nF, Xo);
        const double zp = depth_of(Rpw, tpw, tau, Xo);
        if (zc > A.min_d && zp > A.min_d && zc < A.max_d && zp < A.max_d) {
            tacc[i] = 1;
            tX[3 * i] = Xo[0]; tX[3 * i + 1] = Xo[1]; tX[3 * i + 2] = Xo[2];
        }                                                               // else retained (quirk Q5)
    }
}

// pass 3: ordered append of the accepted candidates to the landmarks, in-place compaction of the rest
VO_DEV void tri_append(const TriArgs& A, TriShared& sh)
{
    __shared__ int lds[16];
    const int b = blockIdx.x, tid = threadIdx.x;
    const vo_dims& d = A.d;
    const vo_state& s = A.s;
    const int nC = s.nC[b];
    float* ck = s.c_kp + (int64_t)b * d.pcap * 2;
    float* cf = s.c_first + (int64_t)b * d.pcap * 2;
    int32_t* ct = s.c_tau + (int64_t)b * d.pcap;
    float* X = s.lm_X + (int64_t)b * d.ncap * 3;
    float* kp = s.lm_kp + (int64_t)b * d.ncap * 2;
    const int kmax = d.ncap > d.pcap ? d.ncap : d.pcap;
    const int32_t* tacc = s.iwork + (int64_t)b * d.iwork_stride + kmax;
    const float* tX = (const float*)(s.work + (int64_t)b * d.work_stride);
    int nL = s.nL[b];
    int kept = 0;
    for (int base = 0; base < nC; base += blockDim.x) {
        const int i = base + tid;
        const int nvalid = nC - base < (int)blockDim.x ? nC - base : (int)blockDim.x;
        const bool valid = i < nC;
        bool accept = false;
        float k0 = 0, k1 = 0, f0 = 0, f1 = 0;
        int tau = 0;
        if (valid) {
            k0 = ck[2 * i]; k1 = ck[2 * i + 1]; f0 = cf[2 * i]; f1 = cf[2 * i + 1]; tau = ct[i];
            accept = tacc[i] != 0;
        }
        int tacc_n;
        const int pre = block_scan_flag(accept, lds, &tacc_n);          // every thread before tid is valid
        if (accept) {
            const int pa = nL + pre;
            if (pa < d.ncap) {
                X[3 * pa] = tX[3 * i]; X[3 * pa + 1] = tX[3 * i + 1]; X[3 * pa + 2] = tX[3 * i + 2];
                kp[2 * pa] = k0; kp[2 * pa + 1] = k1;
            } else {
                sh.fail = 1;
            }
        } else if (valid) {
            const int pr = kept + (tid - pre);
            ck[2 * pr] = k0; ck[2 * pr + 1] = k1; cf[2 * pr] = f0; cf[2 * pr + 1] = f1; ct[pr] = tau;
        }
        nL += tacc_n;
        kept += nvalid - tacc_n;
        __syncthreads();
    }
    if (tid == 0) {
        s.nL[b] = nL < d.ncap ? nL : d.ncap;
        s.nC[b] = kept;
        if (sh.fail) s.status[b] = VO_ST_CAPACITY;
    }
}

VO_DEV void triangulate_block(const TriArgs& A)
{
    __shared__ TriShared sh;
    if (!tri_setup(A, sh)) return;
    tri_gate(A, sh);
    PNPPROF(26);
    tri_solve(A, sh, sh.m, threadIdx.x, blockDim.x);
    __syncthreads();
    PNPPROF(27);
    tri_append(A, sh);
}

__global__ void __launch_bounds__(256) k_triangulate(TriArgs A) { triangulate_block(A); }

// vo_triangulate as three launches: the gate (one block per chain, list length into iwork), the
// triangulations over TRI_SPLIT blocks per chain, the ordered append (one block per chain).  With
// few chains the one-block form left most CUs idle while each block ran ~12 serial 4x4 SVDs per
// thread (the bootstrap's ~3,000 candidates per chain).
#define TRI_SPLIT 8
__global__ void __launch_bounds__(256) k_tri_gate(TriArgs A)
{
    __shared__ TriShared sh;
    if (!tri_setup(A, sh)) return;
    tri_gate(A, sh);
    if (threadIdx.x == 0) {
        const int kmax = A.d.ncap > A.d.pcap ? A.d.ncap : A.d.pcap;
        A.s.iwork[(int64_t)blockIdx.x * A.d.iwork_stride + 2 * kmax] = sh.m;
    }
}
__global__ void __launch_bounds__(256) k_tri_solve(TriArgs A)
{
    __shared__ TriShared sh;
    if (!tri_setup(A, sh)) return;
    const int kmax = A.d.ncap > A.d.pcap ? A.d.ncap : A.d.pcap;
    const int m = A.s.iwork[(int64_t)blockIdx.x * A.d.iwork_stride + 2 * kmax];
    tri_solve(A, sh, m, blockIdx.y * blockDim.x + threadIdx.x, gridDim.y * blockDim.x);
}
__global__ void __launch_bounds__(256) k_tri_append(TriArgs A)
{
    __shared__ TriShared sh;
    if (!tri_setup(A, sh)) return;
    tri_append(A, sh);
}

// vo_pnp + vo_triangulate(force 0) as one launch (the engine's step): the triangulation of a
// chain runs in the block that just solved its pose, instead of waiting for CUs again
template <int WPE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, 8)))
k_pnp_tri(PnPArgs A, TriArgs T)
{
    if (T.compact) {                      // the tracking stage left the status filtering to us
        track_compact_block(T.d, T.s);
        __syncthreads();
    }
    __shared__ double defer[12];
    __shared__ int pend;
    if (threadIdx.x == 0) pend = 0;
    pnp_ransac_block(A, defer, &pend);
    __syncthreads();
    pnp_apply_split(T.d, T.s, A.rvec, A.tvec, A.success, A.mask, defer, pend);
    __syncthreads();
    PNPPROF(14);
    triangulate_block(T);
    PNPPROF(15);
}

// ------------------------------------------------ feature adding + step finish
#define ADD_THREADS 1024
#define ADD_MAX_CELLS 8192
#define ADD_MAX_ITEMS 16384

struct AddArgs {
    vo_dims d;
    vo_state s;
    double min_dist;
    int boot;              // 1: bootstrap finish (no GFTT)
};

__global__ void __launch_bounds__(ADD_THREADS) k_add_finish(AddArgs A)
{
    __shared__ int cstart[ADD_MAX_CELLS + 1];
    __shared__ int cfill[ADD_MAX_CELLS];
    __shared__ int items_lds[ADD_MAX_ITEMS];
    __shared__ int lds[16];
    __shared__ int sh_scan[ADD_THREADS / 64];
    const int b = blockIdx.x, tid = threadIdx.x;
    const vo_dims& d = A.d;
    const vo_state& s = A.s;
    if (s.status[b] != 0) return;
    const int nF = s.nF[b];
    const int M = s.nCorners[b];
    if (M < 0) { if (tid == 0) s.status[b] = VO_ST_CAPACITY; return; }      // k_gftt_select overflow
    if (M == 0) { if (tid == 0) s.status[b] = VO_ST_GFTT_NONE; return; }   // None.squeeze()
    if (M == 1) { if (tid == 0) s.status[b] = VO_ST_GFTT_ONE; return; }    // (2,) indexing
    const int P = s.nC[b];
    float* ck = s.c_kp + (int64_t)b * d.pcap * 2;
    float* cf = s.c_first + (int64_t)b * d.pcap * 2;
    int32_t* ct = s.c_tau + (int64_t)b * d.pcap;
    const float* cor = s.corners + (int64_t)b * d.mcap * 2;
    const float mdf = (float)A.min_dist;
    // cells of at least minDistance: the 3x3 neighbourhood holds every candidate within it.
    // Coarser cells keep that exact, so they grow until the grid fits the LDS tables.
    int cs = (int)ceil(A.min_dist) > 0 ? (int)ceil(A.min_dist) : 1;
    while ((d.W / cs + 3) * (d.H / cs + 3) > ADD_MAX_CELLS) ++cs;
    const int gw = d.W / cs + 3, gh = d.H / cs + 3;
    // the cell-sorted candidate list lives in LDS, or for more than ADD_MAX_ITEMS candidates
    // (C5: ~15k points per chain) in the chain's int scratch, free once PnP is done (same
    // stream) -- the all-pairs fallback below is O(M * P)
    int* items = items_lds;
    if (P > ADD_MAX_ITEMS) items = s.iwork + (int64_t)b * d.iwork_stride;
    const bool grid = (gw * gh <= ADD_MAX_CELLS) && (P <= ADD_MAX_ITEMS || P <= d.iwork_stride);
    if (grid) {
        for (int q = tid; q < gw * gh; q += blockDim.x) cfill[q] = 0;
        __syncthreads();
        for (int i = tid; i < P; i += blockDim.x) {
            int cx = (int)floorf(ck[2 * i] / (float)cs) + 1, cy = (int)floorf(ck[2 * i + 1] / (float)cs) + 1;
            cx = cx < 0 ? 0 : (cx > gw - 1 ? gw - 1 : cx);
            cy = cy < 0 ? 0 : (cy > gh - 1 ? gh - 1 : cy);
            atomicAdd(&cfill[cy * gw + cx], 1);
        }
        __syncthreads();
        // exclusive scan of cell counts (block-wide, sequential chunks per thread)
        const int ncell = gw * gh;
        const int per = (ncell + blockDim.x - 1) / blockDim.x;
        int local = 0;
        for (int q = tid * per; q < (tid + 1) * per && q < ncell; ++q) local += cfill[q];
        int incl = local;
        for (int o = 1; o < 64; o <<= 1) { int v = __shfl_up(incl, o, 64); if (lane_id() >= o) incl += v; }
        if (lane_id() == 63) sh_scan[wave_id()] = incl;
        __syncthreads();
        int wbase = 0;
        for (int w = 0; w < wave_id(); ++w) wbase += sh_scan[w];
        int run = wbase + incl - local;
        for (int q = tid * per; q < (tid + 1) * per && q < ncell; ++q) { cstart[q] = run; run += cfill[q]; cfill[q] = 0; }
        if (tid == 0) cstart[ncell] = P;
        __syncthreads();
        for (int i = tid; i < P; i += blockDim.x) {
            int cx = (int)floorf(ck[2 * i] / (float)cs) + 1, cy = (int)floorf(ck[2 * i + 1] / (float)cs) + 1;
            cx = cx < 0 ? 0 : (cx > gw - 1 ? gw - 1 : cx);
            cy = cy < 0 ? 0 : (cy > gh - 1 ? gh - 1 : cy);
            const int cell = cy * gw + cx;
            items[cstart[cell] + atomicAdd(&cfill[cell], 1)] = i;
        }
        __syncthreads();
    }
    int nC = P;
    for (int base = 0; base < M; base += blockDim.x) {
        const int j = base + tid;
        bool keep = false;
        float x = 0, y = 0;
        if (j < M) {
            x = cor[2 * j]; y = cor[2 * j + 1];
            keep = true;
            if (grid) {
                const int cx = (int)floorf(x / (float)cs) + 1, cy = (int)floorf(y / (float)cs) + 1;
                for (int yy = cy - 1; yy <= cy + 1 && keep; ++yy) {
                    if (yy < 0 || yy >= gh) continue;
                    for (int xx = cx - 1; xx <= cx + 1 && keep; ++xx) {
                        if (xx < 0 || xx >= gw) continue;
                        const int cell = yy * gw + xx;
                        for (int q = cstart[cell]; q < cstart[cell + 1]; ++q) {
                            const int i = items[q];
                            const float dx = x - ck[2 * i], dy = y - ck[2 * i + 1];
                            if (!(sqrtf(dx * dx + dy * dy) > mdf)) { keep = false; break; }
                        }
                    }
                }
            } else {
                for (int i = 0; i < P && keep; ++i) {
                    const float dx = x - ck[2 * i], dy = y - ck[2 * i + 1];
                    if (!(sqrtf(dx * dx + dy * dy) > mdf)) keep = false;
                }
            }
        }
        __syncthreads();   // all reads of ck in this chunk done before appends
        int tot;
        const int pos = nC + block_scan_flag(keep, lds, &tot);
        if (keep && pos < d.pcap) {
            ck[2 * pos] = x; ck[2 * pos + 1] = y;
            cf[2 * pos] = x; cf[2 * pos + 1] = y;
            ct[pos] = nF;                                             // tau = len(transforms)
        }
        nC += tot;
        __syncthreads();
    }
    if (tid == 0) {
        if (nC > d.pcap) { s.status[b] = VO_ST_CAPACITY; nC = d.pcap; }
        s.nC[b] = nC;
        s.num_pts[(int64_t)b * d.fcap + nF] = s.nInl[b];
        s.nF[b] = nF + 1;
    }
}

#define ADD_LEAN_THREADS 256
// k_add_finish for many chains per launch (round 5, the headline's 384): a 4-wave block
// whose only LDS is the cell start table (uint16, 16 KB); the per-cell fill counters and the
// cell-sorted candidate list live in the chain's int scratch (free once PnP is done, same
// stream).  The 16-wave, 128 KB-LDS form needed a CU with nearly all of its LDS free, which
// under another stream group's LK flood (~4 KB of LDS per wave) meant waiting for a CU to
// drain (headline 65.7k -> 66.2-66.5k frames/s; at 1-128 chains per launch the
// 16-wave form is faster, 2-5 %: profiles/r5_add_lean_ab.jsonl).  The result does not depend on the block shape: the grid only narrows which existing
// candidates a corner is tested against (any one within min_dist rejects it), and the corners
// are appended in their order by the chunked block scan.
__global__ void __launch_bounds__(ADD_LEAN_THREADS) k_add_finish_lean(AddArgs A)
{
    __shared__ uint16_t cstart[ADD_MAX_CELLS + 1];
    __shared__ int lds[16];
    __shared__ int sh_scan[ADD_LEAN_THREADS / 64];
    const int b = blockIdx.x, tid = threadIdx.x;
    const vo_dims& d = A.d;
    const vo_state& s = A.s;
    if (s.status[b] != 0) return;
    const int nF = s.nF[b];
    const int M = s.nCorners[b];
    if (M < 0) { if (tid == 0) s.status[b] = VO_ST_CAPACITY; return; }      // k_gftt_select overflow
    if (M == 0) { if (tid == 0) s.status[b] = VO_ST_GFTT_NONE; return; }   // None.squeeze()
    if (M == 1) { if (tid == 0) s.status[b] = VO_ST_GFTT_ONE; return; }    // (2,) indexing
    const int P = s.nC[b];
    float* ck = s.c_kp + (int64_t)b * d.pcap * 2;
    float* cf = s.c_first + (int64_t)b * d.pcap * 2;
    int32_t* ct = s.c_tau + (int64_t)b * d.pcap;
    const float* cor = s.corners + (int64_t)b * d.mcap * 2;
    const float mdf = (float)A.min_dist;
    // cells of at least minDistance: the 3x3 neighbourhood holds every candidate within it.
    // Coarser cells keep that exact, so they grow until the grid fits the LDS table.
    int cs = (int)ceil(A.min_dist) > 0 ? (int)ceil(A.min_dist) : 1;
    while ((d.W / cs + 3) * (d.H / cs + 3) > ADD_MAX_CELLS) ++cs;
    const int gw = d.W / cs + 3, gh = d.H / cs + 3;
    int* cfill = s.iwork + (int64_t)b * d.iwork_stride;                // [ADD_MAX_CELLS]
    int* items = cfill + ADD_MAX_CELLS;                                 // [P]
    // the all-pairs test below (O(M * P)) when the list does not fit the scratch or uint16
    const bool grid = P < 65536 && (int64_t)ADD_MAX_CELLS + P <= d.iwork_stride;
    if (grid) {
        const int ncell = gw * gh;
        for (int q = tid; q < ncell; q += blockDim.x) cfill[q] = 0;
        __syncthreads();
        for (int i = tid; i < P; i += blockDim.x) {
            int cx = (int)floorf(ck[2 * i] / (float)cs) + 1, cy = (int)floorf(ck[2 * i + 1] / (float)cs) + 1;
            cx = cx < 0 ? 0 : (cx > gw - 1 ? gw - 1 : cx);
            cy = cy < 0 ? 0 : (cy > gh - 1 ? gh - 1 : cy);
            atomicAdd(&cfill[cy * gw + cx], 1);
        }
        __syncthreads();
        // exclusive scan of the cell counts (block-wide, sequential chunks per thread)
        const int per = (ncell + blockDim.x - 1) / blockDim.x;
        const int q0 = tid * per, q1 = min(q0 + per, ncell);
        int local = 0;
        for (int q = q0; q < q1; ++q) local += cfill[q];
        int incl = local;
        for (int o = 1; o < 64; o <<= 1) { int v = __shfl_up(incl, o, 64); if (lane_id() >= o) incl += v; }
        if (lane_id() == 63) sh_scan[wave_id()] = incl;
        __syncthreads();
        int wbase = 0;
        for (int w = 0; w < wave_id(); ++w) wbase += sh_scan[w];
        int run = wbase + incl - local;
        for (int q = q0; q < q1; ++q) { const int c = cfill[q]; cstart[q] = (uint16_t)run; run += c; cfill[q] = 0; }
        if (tid == 0) cstart[ncell] = (uint16_t)P;
        __syncthreads();
        for (int i = tid; i < P; i += blockDim.x) {
            int cx = (int)floorf(ck[2 * i] / (float)cs) + 1, cy = (int)floorf(ck[2 * i + 1] / (float)cs) + 1;
            cx = cx < 0 ? 0 : (cx > gw - 1 ? gw - 1 : cx);
            cy = cy < 0 ? 0 : (cy > gh - 1 ? gh - 1 : cy);
            const int cell = cy * gw + cx;
            items[cstart[cell] + atomicAdd(&cfill[cell], 1)] = i;
        }
        __syncthreads();
    }
    int nC = P;
    for (int base = 0; base < M; base += blockDim.x) {
        const int j = base + tid;
        bool keep = false;
        float x = 0, y = 0;
        if (j < M) {
            x = cor[2 * j]; y = cor[2 * j + 1];
            keep = true;
            if (grid) {
                const int cx = (int)floorf(x / (float)cs) + 1, cy = (int)floorf(y / (float)cs) + 1;
                for (int yy = cy - 1; yy <= cy + 1 && keep; ++yy) {
                    if (yy < 0 || yy >= gh) continue;
                    for (int xx = cx - 1; xx <= cx + 1 && keep; ++xx) {
                        if (xx < 0 || xx >= gw) continue;
                        const int cell = yy * gw + xx;
                        for (int q = cstart[cell]; q < cstart[cell + 1]; ++q) {
                            const int i = items[q];
                            const float dx = x - ck[2 * i], dy = y - ck[2 * i + 1];
                            if (!(sqrtf(dx * dx + dy * dy) > mdf)) { keep = false; break; }
                        }
                    }
                }
            } else {
                for (int i = 0; i < P && keep; ++i) {
                    const float dx = x - ck[2 * i], dy = y - ck[2 * i + 1];
                    if (!(sqrtf(dx * dx + dy * dy) > mdf)) keep = false;
                }
            }
        }
        __syncthreads();   // all reads of ck in this chunk done before appends
        int tot;
        const int pos = nC + block_scan_flag(keep, lds, &tot);
        if (keep && pos < d.pcap) {
            ck[2 * pos] = x; ck[2 * pos + 1] = y;
            cf[2 * pos] = x; cf[2 * pos + 1] = y;
            ct[pos] = nF;                                             // tau = len(transforms)
        }
        nC += tot;
        __syncthreads();
    }
    if (tid == 0) {
        if (nC > d.pcap) { s.status[b] = VO_ST_CAPACITY; nC = d.pcap; }
        s.nC[b] = nC;
        s.num_pts[(int64_t)b * d.fcap + nF] = s.nInl[b];
        s.nF[b] = nF + 1;
    }
}

// cv2.triangulatePoints over independent (P1, P2, x1, x2) rows
__global__ void k_tri_points(int n, const double* P1, const double* P2, const float* x1, const float* x2, float* out)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double X4[4];
    tri_one(P1 + 12 * i, P2 + 12 * i, x1[2 * i], x1[2 * i + 1], x2[2 * i], x2[2 * i + 1], X4);
    for (int q = 0; q < 4; ++q) out[4 * i + q] = (float)X4[q];
}

__global__ void k_rodrigues(int n, int to_matrix, const double* in, double* out)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (to_matrix) rodrigues_v2m(in + 3 * i, out + 9 * i);
    else rodrigues_m2v(in + 9 * i, out + 3 * i);
}

}  // namespace

// ======================================================================= host side
#define VO_STREAM(s) ((hipStream_t)(s))
static inline int hip_rc() { return hipGetLastError() == hipSuccess ? VO_OK : VO_EHIP; }

static void fill_pnp(PnPArgs& P, const vo_opts* o)
{
    for (int i = 0; i < 9; ++i) P.K[i] = o->K[i];
    P.thr = (float)(o->pnp_error * o->pnp_error);
    P.conf = o->pnp_conf;
    P.iters = o->pnp_iters;
}

extern "C" int vo_pnp_ransac(const vo_opts* o, int B, const float* obj, const float* img, const int32_t* counts,
                             int32_t cap, double* rvec, double* tvec, int32_t* success, uint8_t* inl_mask,
                             int32_t* n_inl, double* work, int64_t work_stride, vo_stream_t stream)
{
    if (!o || B < 1 || !obj || !img || !counts || !rvec || !tvec || !success || !inl_mask || !n_inl || !work) return VO_EARG;
    if (work_stride < 12LL * cap + 64) return VO_EARG;
    PnPArgs P;
    fill_pnp(P, o);
    P.min_points = 4;
    P.obj = obj; P.img = img; P.counts = counts; P.cap = cap; P.chain_status = nullptr;
    P.work = work; P.work_stride = work_stride; P.iwork = nullptr; P.iwork_stride = 0;
    P.rvec = rvec; P.tvec = tvec; P.success = success; P.mask = inl_mask; P.n_inl = n_inl;
    hipLaunchKernelGGL(k_pnp_ransac, dim3(B), dim3(256), 0, VO_STREAM(stream), P);
    return hip_rc();
}

static void fill_pnp_engine(PnPArgs& P, const vo_dims* d, const vo_opts* o, const vo_state* s)
{
    fill_pnp(P, o);
    P.min_points = 8;                                                   // :342
    P.obj = s->lm_X; P.img = s->lm_kp; P.counts = s->nL; P.cap = d->ncap; P.chain_status = s->status;
    P.work = s->work; P.work_stride = d->work_stride; P.iwork = s->iwork; P.iwork_stride = d->iwork_stride;
    P.rvec = s->pnp_rt; P.tvec = s->pnp_rt + 3LL * d->B;
    P.success = s->pnp_ok; P.n_inl = s->pnp_ninl; P.mask = s->pnp_mask;
}

extern "C" int vo_pnp(const vo_dims* d, const vo_opts* o, const vo_state* s, vo_stream_t stream)
{
    if (!d || !o || !s) return VO_EARG;
    if (d->work_stride < 12LL * d->ncap + 64) return VO_EARG;
    PnPArgs P;
    fill_pnp_engine(P, d, o, s);
    hipStream_t st = VO_STREAM(stream);
    static const int split = [] { const char* e = getenv("VO_PNP_SPLIT"); return e ? atoi(e) : 0; }();
    if (split == 1) {                     // the two-launch form (A/B measurements)
        hipLaunchKernelGGL(k_pnp_ransac, dim3(d->B), dim3(256), 0, st, P);
        hipLaunchKernelGGL(k_pnp_apply, dim3(d->B), dim3(256), 0, st, *d, *s, P.rvec, P.tvec, P.success, P.mask);
    } else if (d->B > (device_cus() > 0 ? device_cus() : 256)) {
        // more chains than CUs: two blocks per CU (as vo_pnp_triangulate)
        hipLaunchKernelGGL(k_pnp_fused<VO_PNP_WPE>, dim3(d->B), dim3(256), 0, st, P, *d, *s);
    } else {
        hipLaunchKernelGGL(k_pnp_fused<1>, dim3(d->B), dim3(256), 0, st, P, *d, *s);
    }
    return hip_rc();
}

static void fill_tri(TriArgs& A, const vo_dims* d, const vo_opts* o, const vo_state* s, int force)
{
    A.d = *d;
    A.s = *s;
    for (int i = 0; i < 9; ++i) { A.K[i] = o->K[i]; A.Kinv[i] = o->K_inv[i]; }
    A.min_d = o->min_dist_landmarks;
    A.max_d = o->max_dist_landmarks;
    A.cos_thr = o->cos_baseline;
    A.min_frames = o->min_baseline_frames;
    A.force = force;
    A.compact = 0;
}

extern "C" int vo_triangulate(const vo_dims* d, const vo_opts* o, const vo_state* s, int force, vo_stream_t stream)
{
    if (!d || !o || !s) return VO_EARG;
    TriArgs A;
    fill_tri(A, d, o, s, force);
    const int kmax = d->ncap > d->pcap ? d->ncap : d->pcap;
    if (d->iwork_stride < 2LL * kmax + 1) return VO_EARG;
    hipStream_t st = VO_STREAM(stream);
    if (d->B >= (device_cus() > 0 ? device_cus() : 256)) {
        hipLaunchKernelGGL(k_triangulate, dim3(d->B), dim3(256), 0, st, A);
    } else {
        hipLaunchKernelGGL(k_tri_gate, dim3(d->B), dim3(256), 0, st, A);
        hipLaunchKernelGGL(k_tri_solve, dim3(d->B, TRI_SPLIT), dim3(256), 0, st, A);
        hipLaunchKernelGGL(k_tri_append, dim3(d->B), dim3(256), 0, st, A);
    }
    return hip_rc();
}

static int launch_pnp_tri(const vo_dims* d, const vo_opts* o, const vo_state* s, int compact, vo_stream_t stream)
{
    if (!d || !o || !s) return VO_EARG;
    if (d->work_stride < 12LL * d->ncap + 64) return VO_EARG;
    PnPArgs P;
    fill_pnp_engine(P, d, o, s);
    TriArgs T;
    fill_tri(T, d, o, s, 0);
    T.compact = compact;
    // more chains than CUs: the 2-waves/SIMD build (two blocks per CU, some registers spilled);
    // otherwise every block has a CU of its own and the unconstrained build is faster
    // (VO_PNP_TRI_WPE=1|2 forces one build: measurement option)
    static const int force = [] { const char* e = getenv("VO_PNP_TRI_WPE"); return e ? atoi(e) : 0; }();
    const int n_cu = device_cus() > 0 ? device_cus() : 256;      // of the current device
    const bool two = force ? force == 2 : d->B > n_cu;
    if (two) hipLaunchKernelGGL(k_pnp_tri<VO_PNP_WPE>, dim3(d->B), dim3(256), 0, VO_STREAM(stream), P, T);
    else hipLaunchKernelGGL(k_pnp_tri<1>, dim3(d->B), dim3(256), 0, VO_STREAM(stream), P, T);
    return hip_rc();
}

extern "C" int vo_pnp_triangulate(const vo_dims* d, const vo_opts* o, const vo_state* s, vo_stream_t stream)
{
    return launch_pnp_tri(d, o, s, 0, stream);
}

extern "C" int vo_filter_pnp_triangulate(const vo_dims* d, const vo_opts* o, const vo_state* s, vo_stream_t stream)
{
    return launch_pnp_tri(d, o, s, 1, stream);
}

extern "C" int vo_add_corners_finish(const vo_dims* d, const vo_opts* o, const vo_state* s, vo_stream_t stream)
{
    if (!d || !o || !s) return VO_EARG;
    AddArgs A;
    A.d = *d;
    A.s = *s;
    A.min_dist = o->feature_min_dist;
    A.boot = 0;
    // the lean form from 256 chains per launch (VO_ADD_LEAN=0 / 1 forces it off / on)
    static const int lean_env = [] { const char* e = getenv("VO_ADD_LEAN"); return e ? atoi(e) : -1; }();
    if (lean_env >= 0 ? lean_env == 1 : d->B >= 256)
        hipLaunchKernelGGL(k_add_finish_lean, dim3(d->B), dim3(ADD_LEAN_THREADS), 0, VO_STREAM(stream), A);
    else
        hipLaunchKernelGGL(k_add_finish, dim3(d->B), dim3(ADD_THREADS), 0, VO_STREAM(stream), A);
    return hip_rc();
}

namespace {
__global__ void k_status_word(const int32_t* status, const int32_t* n_inl, int32_t* dst)
{
    if (threadIdx.x == 0) { dst[0] = status[0]; dst[1] = n_inl[0]; }
}
}  // namespace

extern "C" int vo_status_word(const vo_state* s, int32_t* dst, vo_stream_t stream)
{
    if (!s || !dst) return VO_EARG;
    hipLaunchKernelGGL(k_status_word, dim3(1), dim3(64), 0, VO_STREAM(stream), s->status, s->nInl, dst);
    return hip_rc();
}

extern "C" int vo_triangulate_points(int n, const double* P1, const double* P2, const float* x1, const float* x2,
                                     float* out4, vo_stream_t stream)
{
    if (n < 0 || (n > 0 && (!P1 || !P2 || !x1 || !x2 || !out4))) return VO_EARG;
    if (n == 0) return VO_OK;
    hipLaunchKernelGGL(k_tri_points, dim3((n + 127) / 128), dim3(128), 0, VO_STREAM(stream), n, P1, P2, x1, x2, out4);
    return hip_rc();
}

extern "C" int vo_rodrigues(int n, int to_matrix, const double* in, double* out, vo_stream_t stream)
{
    if (n < 0 || (n > 0 && (!in || !out))) return VO_EARG;
    if (n == 0) return VO_OK;
    hipLaunchKernelGGL(k_rodrigues, dim3((n + 127) / 128), dim3(128), 0, VO_STREAM(stream), n, to_matrix, in, out);
    return hip_rc();
}
