// Device helpers shared by the gfx950 kernels of libvo_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/vo_hip.h"

#define VO_DEV __device__ __forceinline__

VO_DEV int lane_id() { return threadIdx.x & 63; }
VO_DEV int wave_id() { return threadIdx.x >> 6; }

// BORDER_REFLECT_101 index (cv::borderInterpolate)
VO_DEV int refl101(int p, int len)
{
    if (len == 1) return 0;
    while (p < 0 || p >= len) p = (p < 0) ? -p : 2 * len - p - 2;
    return p;
}

VO_DEV int64_t wave_sum_i64(int64_t v)
{
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

VO_DEV int wave_sum_i32(int v)
{
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Wave-wide int32 sum with DPP (VALU lane moves, no LDS crossbar): quad swaps, row
// rotations, then the GFX9 row broadcasts; lane 63 ends with the total.
VO_DEV int wave_sum_dpp(int x)
{
    x += __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    x += __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    x += __builtin_amdgcn_update_dpp(0, x, 0x124, 0xF, 0xF, false);  // row_ror:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x128, 0xF, 0xF, false);  // row_ror:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);  // row_bcast:15
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return __builtin_amdgcn_readlane(x, 63);
}

// Two wave sums with their DPP steps interleaved: each step's two adds are independent, so the
// chain issues back to back instead of waiting out the DPP read hazard of one reduction.
VO_DEV void wave_sum2_dpp(int& x, int& y)
{
    x += __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false);
    y += __builtin_amdgcn_update_dpp(0, y, 0xB1, 0xF, 0xF, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false);
    y += __builtin_amdgcn_update_dpp(0, y, 0x4E, 0xF, 0xF, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x124, 0xF, 0xF, false);
    y += __builtin_amdgcn_update_dpp(0, y, 0x124, 0xF, 0xF, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x128, 0xF, 0xF, false);
    y += __builtin_amdgcn_update_dpp(0, y, 0x128, 0xF, 0xF, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);
    y += __builtin_amdgcn_update_dpp(0, y, 0x142, 0xA, 0xF, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);
    y += __builtin_amdgcn_update_dpp(0, y, 0x143, 0xC, 0xF, false);
    x = __builtin_amdgcn_readlane(x, 63);
    y = __builtin_amdgcn_readlane(y, 63);
}

// Two wave sums in one DPP chain: v_permlane32_swap trades the upper half of x for the lower
// half of y, so one add leaves x's half-sums in lanes 0..31 and y's in 32..63; five row-level
// steps finish both (totals in lanes 31 and 63).  Exact for int32 partials whose sums fit.
VO_DEV void wave_sum2_swap(int& x, int& y)
{
    const auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
    int v = (int)r[0] + (int)r[1];
    v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    v += __builtin_amdgcn_update_dpp(0, v, 0x124, 0xF, 0xF, false);  // row_ror:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x128, 0xF, 0xF, false);  // row_ror:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    x = __builtin_amdgcn_readlane(v, 31);
    y = __builtin_amdgcn_readlane(v, 63);
}

// Three wave sums: x and y share one chain through the half swap (as wave_sum2_swap), z runs
// its own six steps interleaved with it.
VO_DEV void wave_sum3_swap(int& x, int& y, int& z)
{
    const auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
    int v = (int)r[0] + (int)r[1];
#define VO_DPP2(ctl, rm) \
    v += __builtin_amdgcn_update_dpp(0, v, ctl, rm, 0xF, false); \
    z += __builtin_amdgcn_update_dpp(0, z, ctl, rm, 0xF, false);
    VO_DPP2(0xB1, 0xF) VO_DPP2(0x4E, 0xF) VO_DPP2(0x124, 0xF) VO_DPP2(0x128, 0xF) VO_DPP2(0x142, 0xA)
#undef VO_DPP2
    z += __builtin_amdgcn_update_dpp(0, z, 0x143, 0xC, 0xF, false);
    x = __builtin_amdgcn_readlane(v, 31);
    y = __builtin_amdgcn_readlane(v, 63);
    z = __builtin_amdgcn_readlane(z, 63);
}

VO_DEV void wave_sum3_dpp(int& x, int& y, int& z)
{
#define VO_DPP3(ctl, rm) \
    x += __builtin_amdgcn_update_dpp(0, x, ctl, rm, 0xF, false); \
    y += __builtin_amdgcn_update_dpp(0, y, ctl, rm, 0xF, false); \
    z += __builtin_amdgcn_update_dpp(0, z, ctl, rm, 0xF, false);
    VO_DPP3(0xB1, 0xF) VO_DPP3(0x4E, 0xF) VO_DPP3(0x124, 0xF) VO_DPP3(0x128, 0xF) VO_DPP3(0x142, 0xA) VO_DPP3(0x143, 0xC)
#undef VO_DPP3
    x = __builtin_amdgcn_readlane(x, 63);
    y = __builtin_amdgcn_readlane(y, 63);
    z = __builtin_amdgcn_readlane(z, 63);
}

// Exact wave-wide sum of per-lane int32 partials whose total may exceed 32 bits:
// p = hi * 2^16 + lo with lo in [0, 65535]; both halves sum exactly in int32 over 64 lanes.
VO_DEV int64_t wave_sum_split(int p)
{
    const int lo = p & 0xFFFF, hi = p >> 16;
    return (int64_t)wave_sum_dpp(hi) * 65536 + (int64_t)wave_sum_dpp(lo);
}

// exclusive prefix of a per-thread flag over the whole block; lds must hold 16 ints
VO_DEV int block_scan_flag(bool f, int* lds, int* total)
{
    unsigned long long m = __ballot(f);
    const int lane = lane_id(), w = wave_id(), nw = blockDim.x >> 6;
    int pre = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) lds[w] = __popcll(m);
    __syncthreads();
    int base = 0, tot = 0;
    for (int i = 0; i < nw; ++i) {
        int c = lds[i];
        if (i < w) base += c;
        tot += c;
    }
    __syncthreads();
    *total = tot;
    return base + pre;
}

// exclusive prefix of a per-thread count over the whole block; lds must hold 16 ints
VO_DEV int block_scan_i32(int v, int* lds, int* total)
{
    const int lane = lane_id(), w = wave_id(), nw = blockDim.x >> 6;
    int inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
    }
    if (lane == 63) lds[w] = inc;
    __syncthreads();
    int base = 0, tot = 0;
    for (int i = 0; i < nw; ++i) {
        const int c = lds[i];
        if (i < w) base += c;
        tot += c;
    }
    __syncthreads();
    *total = tot;
    return base + inc - v;
}

// Linear block id -> work item such that consecutive items share an XCD: hardware
// dispatch sends block L to XCD L % 8, so item = (L % 8) * per_xcd + L / 8 gives each
// XCD a contiguous range (L2 locality only; results do not depend on the mapping).
VO_DEV int xcd_item(int L, int total)
{
    const int per = (total + 7) >> 3;
    return (L & 7) * per + (L >> 3);
}

// sum of an int over the block; lds must hold 16 ints
VO_DEV int block_sum_i32(int v, int* lds)
{
    v = wave_sum_i32(v);
    if (lane_id() == 0) lds[wave_id()] = v;
    __syncthreads();
    int t = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += lds[i];
    __syncthreads();
    return t;
}

// order-preserving map float -> uint32 (larger float -> larger key)
VO_DEV uint32_t fkey(float f)
{
    uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
VO_DEV float fkey_inv(uint32_t k)
{
    uint32_t u = (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k;
    return __uint_as_float(u);
}

// cv::RNG::next()
VO_DEV uint32_t rng_next(uint64_t& s)
{
    s = (uint64_t)(uint32_t)s * 4164903690ULL + (s >> 32);
    return (uint32_t)s;
}

#define DESCALE(x, n) (((x) + (1 << ((n)-1))) >> (n))

// host: compute units of the current device, cached per device id (launch-shape decisions of
// the C ABI entry points; a benign race only stores the same value twice), or the count set by
// vo_set_launch_cus (test hook: the many-chains forms on a small batch)
extern int vo_launch_cus_override;
static inline int device_cus()
{
    if (vo_launch_cus_override > 0) return vo_launch_cus_override;
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 0;
    static int cache[64] = {0};
    if (dev < 64 && cache[dev] > 0) return cache[dev];
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    if (dev < 64) cache[dev] = n;
    return n;
}

// feature_tracking's filtering (VisualOdometryPipeLine.py:283-290) for chain blockIdx.x: the
// tracked landmarks and candidates with status 1, in order (ordered compaction from the tracking
// scratch trk_pts / trk_st)
VO_DEV void track_compact_block(const vo_dims& d, const vo_state& s)
{
    __shared__ int lds[16];
    const int b = blockIdx.x;
    if (s.status[b] != 0) return;
    const int nL = s.nL[b], nC = s.nC[b];
    const int ocap = d.ncap + d.pcap;
    const float* tp = s.trk_pts + (int64_t)b * ocap * 2;
    const uint8_t* ts = s.trk_st + (int64_t)b * ocap;
    float* X = s.lm_X + (int64_t)b * d.ncap * 3;
    float* kp = s.lm_kp + (int64_t)b * d.ncap * 2;
    int out = 0;
    for (int base = 0; base < nL; base += blockDim.x) {
        const int i = base + threadIdx.x;
        const bool ok = i < nL && ts[i] == 1;
        float x0 = 0, x1 = 0, x2 = 0, k0 = 0, k1 = 0;
        if (ok) { x0 = X[3 * i]; x1 = X[3 * i + 1]; x2 = X[3 * i + 2]; k0 = tp[2 * i]; k1 = tp[2 * i + 1]; }
        int tot;
        const int pos = out + block_scan_flag(ok, lds, &tot);
        if (ok) { X[3 * pos] = x0; X[3 * pos + 1] = x1; X[3 * pos + 2] = x2; kp[2 * pos] = k0; kp[2 * pos + 1] = k1; }
        out += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) s.nL[b] = out;
    if (nC <= 1) return;   // quirk Q7: a single candidate is neither tracked nor filtered
    float* ck = s.c_kp + (int64_t)b * d.pcap * 2;
    float* cf = s.c_first + (int64_t)b * d.pcap * 2;
    int32_t* ct = s.c_tau + (int64_t)b * d.pcap;
    out = 0;
    for (int base = 0; base < nC; base += blockDim.x) {
        const int i = base + threadIdx.x;
        const bool ok = i < nC && ts[nL + i] == 1;
        float k0 = 0, k1 = 0, f0 = 0, f1 = 0;
        int tau = 0;
        if (ok) { k0 = tp[2 * (nL + i)]; k1 = tp[2 * (nL + i) + 1]; f0 = cf[2 * i]; f1 = cf[2 * i + 1]; tau = ct[i]; }
        int tot;
        const int pos = out + block_scan_flag(ok, lds, &tot);
        if (ok) { ck[2 * pos] = k0; ck[2 * pos + 1] = k1; cf[2 * pos] = f0; cf[2 * pos + 1] = f1; ct[pos] = tau; }
        out += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) s.nC[b] = out;
}

