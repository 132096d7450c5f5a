// LGKM_CNT depth probe (tools/lgkm_check.py): what does gfx950 do when a wave
// issues more LDS operations than the 4-bit LGKM counter (0..15) can count, and then waits with
// s_waitcnt lgkmcnt(N)?  If the wave stalls at issue while 15 are outstanding (the counter stays
// exact), the first results are complete at the wait; if the counter saturated instead, the wait
// would release early and the copies below would see the sentinel.
//   mode 0: 20 ds_read_b32 in flight, s_waitcnt lgkmcnt(10), copy results 0..7 (an exact counter
//           guarantees 10 complete) -- the shape of the dropped k_lk_w variant (24 reads,
//           lgkmcnt(14));
//   mode 1: 15 ds_write_b8 + 2 ds_read_b32, s_waitcnt lgkmcnt(1), copy the first read -- the
//           shape lgkm_check reports in k_pyr_level<true,32> / k_pyr01 (17 ops, lgkmcnt(1)).
// conflict = 1 puts every lane of an instruction on one LDS bank (64-way serialisation: long
// latency, so an early release would show).  Prints the number of wrong copies per case.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define SENT 0xDEADBEEFu
#define NLDS (64 * 64 + 128)

__device__ __forceinline__ uint32_t val(uint32_t i) { return i * 2654435761u + 12345u; }

__global__ void __launch_bounds__(64) k_probe0(uint32_t* bad, int conflict, int iters)
{
    __shared__ uint32_t lds[NLDS];
    const int lane = threadIdx.x;
    for (int i = lane; i < NLDS; i += 64) lds[i] = val(i);
    __syncthreads();
    const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)lds;
    const uint32_t row = conflict ? lane * 64u : (uint32_t)lane;
    const uint32_t addr = base + 4u * row;
    uint32_t nbad = 0;
    for (int it = 0; it < iters; ++it) {
        uint32_t c0, c1, c2, c3, c4, c5, c6, c7;
        uint32_t r0 = SENT, r1 = SENT, r2 = SENT, r3 = SENT, r4 = SENT, r5 = SENT, r6 = SENT, r7 = SENT, r8 = SENT,
                 r9 = SENT, r10 = SENT, r11 = SENT, r12 = SENT, r13 = SENT, r14 = SENT, r15 = SENT, r16 = SENT,
                 r17 = SENT, r18 = SENT, r19 = SENT;
        asm volatile("s_waitcnt lgkmcnt(0)\n\t"
                     "ds_read_b32 %8, %28 offset:0\n\t"
                     "ds_read_b32 %9, %28 offset:4\n\t"
                     "ds_read_b32 %10, %28 offset:8\n\t"
                     "ds_read_b32 %11, %28 offset:12\n\t"
                     "ds_read_b32 %12, %28 offset:16\n\t"
                     "ds_read_b32 %13, %28 offset:20\n\t"
                     "ds_read_b32 %14, %28 offset:24\n\t"
                     "ds_read_b32 %15, %28 offset:28\n\t"
                     "ds_read_b32 %16, %28 offset:32\n\t"
                     "ds_read_b32 %17, %28 offset:36\n\t"
                     "ds_read_b32 %18, %28 offset:40\n\t"
                     "ds_read_b32 %19, %28 offset:44\n\t"
                     "ds_read_b32 %20, %28 offset:48\n\t"
                     "ds_read_b32 %21, %28 offset:52\n\t"
                     "ds_read_b32 %22, %28 offset:56\n\t"
                     "ds_read_b32 %23, %28 offset:60\n\t"
                     "ds_read_b32 %24, %28 offset:64\n\t"
                     "ds_read_b32 %25, %28 offset:68\n\t"
                     "ds_read_b32 %26, %28 offset:72\n\t"
                     "ds_read_b32 %27, %28 offset:76\n\t"
                     "s_waitcnt lgkmcnt(10)\n\t"
                     "v_mov_b32 %0, %8\n\t"
                     "v_mov_b32 %1, %9\n\t"
                     "v_mov_b32 %2, %10\n\t"
                     "v_mov_b32 %3, %11\n\t"
                     "v_mov_b32 %4, %12\n\t"
                     "v_mov_b32 %5, %13\n\t"
                     "v_mov_b32 %6, %14\n\t"
                     "v_mov_b32 %7, %15\n\t"
                     "s_waitcnt lgkmcnt(0)"
                     : "=&v"(c0), "=&v"(c1), "=&v"(c2), "=&v"(c3), "=&v"(c4), "=&v"(c5), "=&v"(c6), "=&v"(c7),
                       "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7), "+v"(r8),
                       "+v"(r9), "+v"(r10), "+v"(r11), "+v"(r12), "+v"(r13), "+v"(r14), "+v"(r15), "+v"(r16),
                       "+v"(r17), "+v"(r18), "+v"(r19)
                     : "v"(addr)
                     : "memory");
        const uint32_t c[8] = {c0, c1, c2, c3, c4, c5, c6, c7};
        const uint32_t r[8] = {r0, r1, r2, r3, r4, r5, r6, r7};
        for (int k = 0; k < 8; ++k) nbad += (c[k] != val(row + k)) + (r[k] != val(row + k));
    }
    if (nbad) atomicAdd(bad, nbad);
}

__global__ void __launch_bounds__(64) k_probe1(uint32_t* bad, int conflict, int iters)
{
    __shared__ uint32_t lds[NLDS];
    const int lane = threadIdx.x;
    for (int i = lane; i < NLDS; i += 64) lds[i] = val(i);
    __syncthreads();
    const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)lds;
    // writes: the first 64 x 64 dwords (conflict: every lane in one bank); reads: the tail
    const uint32_t waddr = base + 4u * (conflict ? lane * 64u : (uint32_t)lane);
    const uint32_t rrow = 64u * 64u + (uint32_t)lane;
    const uint32_t raddr = base + 4u * rrow;
    uint32_t nbad = 0;
    for (int it = 0; it < iters; ++it) {
        uint32_t c, r0 = SENT, r1 = SENT;
        const uint32_t v = (uint32_t)(it + lane);
        asm volatile("s_waitcnt lgkmcnt(0)\n\t"
                     "ds_write_b8 %3, %4 offset:0\n\t"
                     "ds_write_b8 %3, %4 offset:1\n\t"
                     "ds_write_b8 %3, %4 offset:2\n\t"
                     "ds_write_b8 %3, %4 offset:3\n\t"
                     "ds_write_b8 %3, %4 offset:4\n\t"
                     "ds_write_b8 %3, %4 offset:5\n\t"
                     "ds_write_b8 %3, %4 offset:6\n\t"
                     "ds_write_b8 %3, %4 offset:7\n\t"
                     "ds_write_b8 %3, %4 offset:8\n\t"
                     "ds_write_b8 %3, %4 offset:9\n\t"
                     "ds_write_b8 %3, %4 offset:10\n\t"
                     "ds_write_b8 %3, %4 offset:11\n\t"
                     "ds_write_b8 %3, %4 offset:12\n\t"
                     "ds_write_b8 %3, %4 offset:13\n\t"
                     "ds_write_b8 %3, %4 offset:14\n\t"
                     "ds_read_b32 %1, %5\n\t"
                     "ds_read_b32 %2, %5 offset:4\n\t"
                     "s_waitcnt lgkmcnt(1)\n\t"
                     "v_mov_b32 %0, %1\n\t"
                     "s_waitcnt lgkmcnt(0)"
                     : "=&v"(c), "+v"(r0), "+v"(r1)
                     : "v"(waddr), "v"(v), "v"(raddr)
                     : "memory");
        nbad += (c != val(rrow)) + (r0 != val(rrow)) + (r1 != val(rrow + 1));
    }
    if (nbad) atomicAdd(bad, nbad);
}

int main(int argc, char** argv)
{
    const int blocks = argc > 1 ? atoi(argv[1]) : 8192, iters = argc > 2 ? atoi(argv[2]) : 64;
    uint32_t* d;
    if (hipMalloc(&d, 4) != hipSuccess) return 1;
    for (int mode = 0; mode < 2; ++mode)
        for (int conflict = 0; conflict < 2; ++conflict) {
            if (hipMemset(d, 0, 4) != hipSuccess) return 1;
            if (mode == 0) hipLaunchKernelGGL(k_probe0, dim3(blocks), dim3(64), 0, 0, d, conflict, iters);
            else hipLaunchKernelGGL(k_probe1, dim3(blocks), dim3(64), 0, 0, d, conflict, iters);
            uint32_t h = 0;
            if (hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
            printf("{\"mode\": %d, \"conflict\": %d, \"blocks\": %d, \"iters\": %d, \"wrong_copies\": %u}\n",
                   mode, conflict, blocks, iters, h);
        }
    return 0;
}
