// Which A/B lane map does v_mfma_i32_32x32x32_i8 use on gfx950?  Exact integer data,
// asymmetric matrices; prints the mismatch count per hypothesis.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
__global__ void k(const v4i* a, const v4i* b, int* c)
{
    v16i acc = {};
    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[threadIdx.x], b[threadIdx.x], acc, 0, 0, 0);
    for (int r = 0; r < 16; ++r) c[threadIdx.x * 16 + r] = acc[r];
}
int main()
{
    int8_t A[32][32], B[32][32];   // A[i][k], B[k][j]
    srand(3);
    for (int i = 0; i < 32; ++i) for (int k2 = 0; k2 < 32; ++k2) { A[i][k2] = (int8_t)(rand() % 255 - 127); B[i][k2] = (int8_t)(rand() % 255 - 127); }
    int C[32][32];
    for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) { int s = 0; for (int q = 0; q < 32; ++q) s += A[i][q] * B[q][j]; C[i][j] = s; }
    v4i *da, *db; int* dc;
    hipMalloc(&da, 64 * 16); hipMalloc(&db, 64 * 16); hipMalloc(&dc, 64 * 16 * 4);
    for (int hyp = 0; hyp < 2; ++hyp) {
        int8_t ha[64][16], hb[64][16];
        for (int l = 0; l < 64; ++l) {
            const int r = l & 31, h = l >> 5;
            for (int j = 0; j < 16; ++j) {
                const int kk = hyp == 0 ? 16 * h + j : (j < 8 ? 8 * h + j : 16 + 8 * h + (j - 8));
                ha[l][j] = A[r][kk];
                hb[l][j] = B[kk][r];
            }
        }
        hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
        hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, dc);
        int hc[64][16];
        hipMemcpy(hc, dc, sizeof hc, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int l = 0; l < 64; ++l)
            for (int reg = 0; reg < 16; ++reg) {
                const int col = l & 31, row = (reg & 3) + 8 * (reg >> 2) + 4 * (l >> 5);
                bad += hc[l][reg] != C[row][col];
            }
        printf("hypothesis %d (%s): %d / 1024 mismatches\n", hyp, hyp == 0 ? "k = 16h + j" : "k = 8h + j | 16 + 8h + j-8", bad);
    }
    return 0;
}
