// Dependent-chain latency of fp64 operations on one lane of one wave (gfx950), in ns per op
// (100 MHz wall clock over 20,000 dependent operations).  Calibrates the PnP serial-chain
// estimates in DESIGN.md.  build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off f64_latency.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#define N 20000
__global__ void k_lat(double a, double b, double* out, long long* t)
{
    if (threadIdx.x != 0) return;
    double x = a;
    long long t0, t1;
    // 0: mul+add (contract off)
    t0 = wall_clock64();
    for (int i = 0; i < N; ++i) x = x * a + b;
    t1 = wall_clock64(); t[0] = t1 - t0; out[0] = x;
    // 1: fma
    x = a; t0 = wall_clock64();
    for (int i = 0; i < N; ++i) x = __builtin_fma(x, a, b);
    t1 = wall_clock64(); t[1] = t1 - t0; out[1] = x;
    // 2: division
    x = a; t0 = wall_clock64();
    for (int i = 0; i < N; ++i) x = b / x + 1.0;
    t1 = wall_clock64(); t[2] = t1 - t0; out[2] = x;
    // 3: sqrt
    x = a; t0 = wall_clock64();
    for (int i = 0; i < N; ++i) x = sqrt(x) + 1.0;
    t1 = wall_clock64(); t[3] = t1 - t0; out[3] = x;
    // 4: add only
    x = a; t0 = wall_clock64();
    for (int i = 0; i < N; ++i) x = x + b;
    t1 = wall_clock64(); t[4] = t1 - t0; out[4] = x;
    // 5: f32 fma for reference
    float y = (float)a; t0 = wall_clock64();
    for (int i = 0; i < N; ++i) y = __builtin_fmaf(y, (float)a, (float)b);
    t1 = wall_clock64(); t[5] = t1 - t0; out[5] = y;
}
int main()
{
    double* d; long long* t;
    hipMalloc(&d, 64); hipMalloc(&t, 64);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, 0.999999, 1e-7, d, t);
        hipDeviceSynchronize();
    }
    long long h[6];
    hipMemcpy(h, t, sizeof(h), hipMemcpyDeviceToHost);
    const char* nm[6] = {"mul+add", "fma", "div+add", "sqrt+add", "add", "f32 fma"};
    for (int i = 0; i < 6; ++i) printf("%-10s %.2f ns per iteration\n", nm[i], h[i] * 10.0 / N);
    return 0;
}
