// Phase timing of k_gftt_select for one chain with real candidate keys (KITTI frame):
// build with -DVO_SELECT_PROF; keys from tools/micro/keys*.bin (written by a host script).
#include "../../monocular_visual_odometry_va4mr_amd/csrc/vo_image.hip"
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

int main()
{
    long long hdr[4];
    FILE* f = fopen("tools/micro/keys_hdr.bin", "rb");
    if (!f || fread(hdr, 8, 4, f) != 4) { printf("no keys\n"); return 1; }
    fclose(f);
    const int n = (int)hdr[0], W = (int)hdr[1], H = (int)hdr[2];
    const uint32_t mx = (uint32_t)hdr[3];
    std::vector<uint64_t> keys(n);
    f = fopen("tools/micro/keys.bin", "rb");
    if (fread(keys.data(), 8, n, f) != (size_t)n) return 1;
    fclose(f);
    const int ccap = W * H / 2 + 1024, mcap = 1400;
    uint64_t* dk; int32_t *dn, *dnc, *dst; uint32_t *dmax, *dgrid; float* dcor;
    CK(hipMalloc(&dk, 8 * (size_t)ccap)); CK(hipMalloc(&dn, 4)); CK(hipMalloc(&dnc, 4)); CK(hipMalloc(&dst, 4));
    CK(hipMalloc(&dmax, 4)); CK(hipMalloc(&dgrid, 4 * (size_t)W * H)); CK(hipMalloc(&dcor, 8 * mcap));
    SelParams S;
    S.keys = dk; S.nkeys = dn; S.eig_max = dmax; S.quality = 0.1; S.ccap = ccap; S.W = W; S.H = H;
    S.max_corners = 1400; S.min_dist = 10; S.corners = dcor; S.ncorners = dnc; S.mcap = mcap;
    S.gscratch = dgrid; S.gstride = (int64_t)W * H; S.chain_status = dst;
    S.acc_lds = mcap; S.grid_lds = ((W + 9) / 10) * ((H + 9) / 10);
    const size_t lds = 16 * (size_t)PAGE + 4 * (size_t)S.acc_lds + 8 * (size_t)S.grid_lds;
    CK(hipFuncSetAttribute((const void*)k_gftt_select<SEL_THREADS>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<float> ref(2 * 1400);
    {
        FILE* fr = fopen("tools/micro/keys_ref.bin", "rb");
        if (fr) { size_t got = fread(ref.data(), 4, ref.size(), fr); (void)got; fclose(fr); }
    }
    for (int rep = 0; rep < 4; ++rep) {
        CK(hipMemcpy(dk, keys.data(), 8 * (size_t)n, hipMemcpyHostToDevice));
        CK(hipMemcpy(dn, &n, 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(dmax, &mx, 4, hipMemcpyHostToDevice));
        CK(hipMemset(dst, 0, 4));
        { long long z[16] = {0}; CK(hipMemcpyToSymbol(HIP_SYMBOL(g_selprof), z, sizeof z)); }
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_gftt_select<SEL_THREADS>, dim3(1), dim3(SEL_THREADS), lds, 0, S);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        long long t[16];
        CK(hipMemcpyFromSymbol(t, HIP_SYMBOL(g_selprof), sizeof t));
        int nc, np; CK(hipMemcpy(&nc, dnc, 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(&np, dn, 4, hipMemcpyDeviceToHost));
        std::vector<float> cor(2 * mcap);
        CK(hipMemcpy(cor.data(), dcor, 8 * mcap, hipMemcpyDeviceToHost));
        int mism = 0;
        for (int i = 0; i < 2 * nc && i < (int)ref.size(); ++i) mism += cor[i] != ref[i];
        printf("mismatches vs oracle corners: %d, rounds %lld | build+conflicts %.1f us, resolve %.1f us, emit %.1f us\n", mism, t[10],
               (t[5] - t[3]) / 100.0, (t[6] - t[5]) / 100.0, (t[4] - t[6]) / 100.0);
        printf("select: %.3f ms, %d passing, %d corners | compact %.1f us, gather %.1f us, sort %.1f us, greedy %.1f us (100 MHz clock)\n",
               ms, np, nc, (t[1] - t[0]) / 100.0, (t[2] - t[1]) / 100.0, (t[3] - t[2]) / 100.0, (t[4] - t[3]) / 100.0);
    }
    return 0;
}
