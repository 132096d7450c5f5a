// Lane map of v_permlane32_swap_b32 through __builtin_amdgcn_permlane32_swap on gfx950:
// x = lane, y = 100 + lane; prints both returned registers for lanes 0, 31, 32, 63.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* o)
{
    const int l = threadIdx.x;
    const auto r = __builtin_amdgcn_permlane32_swap(l, 100 + l, false, false);
    o[l] = r[0];
    o[64 + l] = r[1];
}
int main()
{
    int* d;
    int h[128];
    if (hipMalloc(&d, 512) != hipSuccess) return 1;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, 512, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    for (int l : {0, 1, 31, 32, 33, 63}) printf("lane %2d: r0 %3d r1 %3d\n", l, h[l], h[64 + l]);
    return 0;
}
