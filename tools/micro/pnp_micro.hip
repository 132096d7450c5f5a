// Micro-benchmark of the PnP building blocks on one CU (latency, not throughput):
// svd_jacobi<12,12> and p3p_solve4 on one thread, epnp_block on one block, and the
// whole k_pnp_ransac for a single chain.  Build: make -C tools/micro; run on the GPU box.
#include "../../monocular_visual_odometry_va4mr_amd/csrc/vo_pose.hip"
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <vector>

__global__ void k_t_svd(const double* Min, double* out, long long* t)
{
    __shared__ double A[144], w[12], V[144];
    for (int i = threadIdx.x; i < 144; i += 64) A[i] = Min[i];
    __syncthreads();
    long long c0 = clock64();
    { __shared__ double cs[18]; vg::svd_jacobi_wave_rr<12, 12>(A, w, V, cs); }
    long long c1 = clock64();
    if (threadIdx.x == 0) {
        t[0] = c1 - c0;
        for (int i = 0; i < 12; ++i) out[i] = w[i];
    }
}

__global__ void k_t_p3p(const double* K, const double* o, const double* im, double* out, long long* t)
{
    if (threadIdx.x != 0) return;
    vg::CamK k = vg::camk(K);
    double R[9], tt[3], oo[12], ii[8];
    for (int i = 0; i < 12; ++i) oo[i] = o[i];
    for (int i = 0; i < 8; ++i) ii[i] = im[i];
    long long c0 = clock64();
    int ok = vg::p3p_solve4(k, oo, ii, R, tt);
    long long c1 = clock64();
    t[0] = c1 - c0;
    out[0] = ok; out[1] = tt[0];
}

__global__ void __launch_bounds__(256) k_t_epnp(const double* K, const double* pws, const double* us, double* alphas,
                                                double* pcs, int n, double* out, long long* t)
{
    __shared__ EpnpShared S;
    __shared__ double R[9], tt[3];
    long long c0 = clock64();
    epnp_block(S, K, pws, us, alphas, pcs, n, R, tt);
    long long c1 = clock64();
    if (threadIdx.x == 0) { t[0] = c1 - c0; for (int i = 0; i < 9; ++i) out[i] = R[i]; }
}


// P3P pieces on lane 0 (wall clock, 100 MHz) and the 64-lane layouts of k_pnp_ransac
__global__ void k_t_p3p_parts(const double* K, const double* pws, const double* us, int n, long long* t)
{
    vg::CamK k = vg::camk(K);
    const int lane = threadIdx.x;
    double o[12], im[8], R[9], T[3], e;
    auto load = [&](int h) {
        for (int j = 0; j < 4; ++j) {
            const int id = (h * 37 + j * 101 + 5) % n;
            for (int q = 0; q < 3; ++q) o[3 * j + q] = pws[3 * id + q];
            for (int q = 0; q < 2; ++q) im[2 * j + q] = us[2 * id + q];
        }
    };
    // lanes 0..3 (one hypothesis' quad): serial lengths (quartic) on each, then one solution
    // per lane (the quad-cooperative root finder needs all four lanes)
    if (lane < 4) {
        load(0);
        double dist[3] = {1.0, 1.2, 0.9}, cs[3] = {0.99, 0.98, 0.985}, L[4][3];
        long long a0 = wall_clock64();
        int ns = vg::p3p_lengths(L, dist, cs);
        long long a1 = wall_clock64();
        int ok = vg::p3p_solution(k, o, im, lane, R, T, &e);
        long long a2 = wall_clock64();
        int ok2 = vg::p3p_solve4(k, o, im, R, T);
        long long a3 = wall_clock64();
        if (lane == 0) { t[0] = a1 - a0; t[1] = a2 - a1; t[2] = a3 - a2; t[3] = ns + 10 * ok + 100 * ok2; }
    }
    __syncthreads();
    // 64 lanes, one hypothesis each, serial solutions (old layout)
    load(lane);
    long long b0 = wall_clock64();
    int ok = vg::p3p_solve4(k, o, im, R, T);
    __syncthreads();
    long long b1 = wall_clock64();
    // 16 hypotheses x 4 solution lanes (new layout)
    load(lane >> 2);
    int ok2 = vg::p3p_solution(k, o, im, lane & 3, R, T, &e);
    __syncthreads();
    long long b2 = wall_clock64();
    if (lane == 0) { t[4] = b1 - b0; t[5] = b2 - b1; t[6] = ok + ok2; }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv)
{
    const int outl_pct = argc > 1 ? atoi(argv[1]) : 10;
    const int n = 700;
    double K[9] = {718.856, 0, 607.1928, 0, 718.856, 185.2157, 0, 0, 1};
    std::vector<double> pws(3 * n), us(2 * n);
    std::vector<float> objf(3 * n), imgf(2 * n);
    srand(1);
    auto U = [](double a, double b) { return a + (b - a) * (rand() / (double)RAND_MAX); };
    for (int i = 0; i < n; ++i) {
        double X = U(-10, 10), Y = U(-2, 2), Z = U(5, 60);
        pws[3 * i] = X; pws[3 * i + 1] = Y; pws[3 * i + 2] = Z;
        double u = K[0] * (X + 0.1) / (Z + 1.0) + K[2], v = K[4] * Y / (Z + 1.0) + K[5];
        if (i % 100 < outl_pct) { u += U(20, 60); v -= U(20, 60); }
        us[2 * i] = u; us[2 * i + 1] = v;
        objf[3 * i] = X; objf[3 * i + 1] = Y; objf[3 * i + 2] = Z;
        imgf[2 * i] = u; imgf[2 * i + 1] = v;
    }
    double M[144];
    for (int a = 0; a < 12; ++a) for (int b = 0; b < 12; ++b) M[a * 12 + b] = 0;
    for (int r = 0; r < 40; ++r) { double v[12]; for (int a = 0; a < 12; ++a) v[a] = U(-1, 1); for (int a = 0; a < 12; ++a) for (int b = 0; b < 12; ++b) M[a * 12 + b] += v[a] * v[b]; }
    double *dM, *dout, *dK, *dp, *du, *dal, *dpc, *dob, *dim;
    long long* dt;
    CK(hipMalloc(&dM, 144 * 8)); CK(hipMalloc(&dout, 64 * 8)); CK(hipMalloc(&dK, 72)); CK(hipMalloc(&dt, 64));
    CK(hipMalloc(&dp, 3 * n * 8)); CK(hipMalloc(&du, 2 * n * 8)); CK(hipMalloc(&dal, 4 * n * 8)); CK(hipMalloc(&dpc, 3 * n * 8));
    CK(hipMalloc(&dob, 12 * 8)); CK(hipMalloc(&dim, 8 * 8));
    CK(hipMemcpy(dM, M, 144 * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dK, K, 72, hipMemcpyHostToDevice));
    CK(hipMemcpy(dp, pws.data(), 3 * n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(du, us.data(), 2 * n * 8, hipMemcpyHostToDevice));
    double o4[12], i4[8];
    for (int j = 0; j < 4; ++j) { for (int q = 0; q < 3; ++q) o4[3 * j + q] = pws[3 * (j * 7 + 1) + q]; for (int q = 0; q < 2; ++q) i4[2 * j + q] = us[2 * (j * 7 + 1) + q]; }
    CK(hipMemcpy(dob, o4, 96, hipMemcpyHostToDevice));
    CK(hipMemcpy(dim, i4, 64, hipMemcpyHostToDevice));
    long long t;
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_t_svd, dim3(1), dim3(64), 0, 0, dM, dout, dt);
        CK(hipDeviceSynchronize()); CK(hipMemcpy(&t, dt, 8, hipMemcpyDeviceToHost));
        printf("svd_jacobi_wave<12,12>: %lld cycles\n", t);
        hipLaunchKernelGGL(k_t_p3p, dim3(1), dim3(64), 0, 0, dK, dob, dim, dout, dt);
        CK(hipDeviceSynchronize()); CK(hipMemcpy(&t, dt, 8, hipMemcpyDeviceToHost));
        printf("p3p_solve4 thread0: %lld cycles\n", t);
        hipLaunchKernelGGL(k_t_epnp, dim3(1), dim3(256), 0, 0, dK, dp, du, dal, dpc, n, dout, dt);
        CK(hipDeviceSynchronize()); CK(hipMemcpy(&t, dt, 8, hipMemcpyDeviceToHost));
        printf("epnp_block n=%d: %lld cycles\n", n, t);
    }
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_t_p3p_parts, dim3(1), dim3(64), 0, 0, dK, dp, du, n, dt);
        long long tt[8]; CK(hipDeviceSynchronize()); CK(hipMemcpy(tt, dt, 64, hipMemcpyDeviceToHost));
        printf("p3p parts (us): lengths %.2f, solution0 %.2f, solve4 %.2f (flags %lld) | wave: 64 hyps serial-solutions %.2f, 16x4 lanes %.2f\n",
               tt[0] / 100.0, tt[1] / 100.0, tt[2] / 100.0, tt[3], tt[4] / 100.0, tt[5] / 100.0);
    }
    // whole RANSAC for one chain
    float *dobj, *dimg; int32_t *dcnt, *dsucc, *dninl; uint8_t* dmask; double *dwork, *drv, *dtv; int32_t* diw;
    CK(hipMalloc(&dobj, 3 * n * 4)); CK(hipMalloc(&dimg, 2 * n * 4)); CK(hipMalloc(&dcnt, 4)); CK(hipMalloc(&dsucc, 4));
    CK(hipMalloc(&dninl, 4)); CK(hipMalloc(&dmask, n)); CK(hipMalloc(&dwork, 16 * n * 8)); CK(hipMalloc(&drv, 24)); CK(hipMalloc(&dtv, 24));
    CK(hipMalloc(&diw, 4 * n * 4));
    CK(hipMemcpy(dobj, objf.data(), 3 * n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dimg, imgf.data(), 2 * n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dcnt, &n, 4, hipMemcpyHostToDevice));
    PnPArgs A;
    for (int i = 0; i < 9; ++i) A.K[i] = K[i];
    A.thr = 64.f; A.conf = 0.99; A.iters = 500; A.min_points = 4;
    A.obj = dobj; A.img = dimg; A.counts = dcnt; A.cap = n; A.chain_status = nullptr;
    A.work = dwork; A.work_stride = 16 * n; A.iwork = diw; A.iwork_stride = 4 * n;
    A.rvec = drv; A.tvec = dtv; A.success = dsucc; A.mask = dmask; A.n_inl = dninl;
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_pnp_ransac, dim3(1), dim3(256), 0, 0, A);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        int ni; CK(hipMemcpy(&ni, dninl, 4, hipMemcpyDeviceToHost));
        printf("k_pnp_ransac 1 chain n=%d: %.3f ms, inliers %d\n", n, ms, ni);
        long long t[32];
        CK(hipMemcpyFromSymbol(t, HIP_SYMBOL(g_pnpprof), sizeof t));
        printf("  (us) sample %.1f P3P %.1f, score+update %.1f [last chunk], epnp: mtm %.1f svd12 %.1f betas %.1f R_and_t x3 %.1f | ransac total %.1f compaction %.1f epnp %.1f\n",
               (t[6] - t[1]) / 100.0, (t[2] - t[6]) / 100.0, (t[3] - t[2]) / 100.0, (t[10] - t[4]) / 100.0 + 0 * (t[11] - t[10]), (t[11] - t[10]) / 100.0,
               (t[12] - t[11]) / 100.0, (t[13] - t[12]) / 100.0, (t[3] - t[0]) / 100.0, (t[4] - t[3]) / 100.0, (t[5] - t[4]) / 100.0);
    }
    return 0;
}
