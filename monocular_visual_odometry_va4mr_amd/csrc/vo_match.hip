// Batched brute-force 2-NN matcher on MFMA (cv2.BFMatcher().knnMatch(d0, d1, k=2),
// /root/reference/VisualOdometryPipeLine.py:36,229; SURVEY.md §8a row a4, §8d "BF kNN").
//
// B independent (query set, train set) problems per launch.  SIFT descriptors hold integers
// 0..255, so the squared distances are exact integers and OpenCV's float path (sum < 2^24,
// then sqrtf) is reproduced bit for bit from them.
//
// Default path, int8 (v_mfma_i32_32x32x32_i8, twice the bf16 rate):
//  k_bf_prep_i8  descriptors -> int8 rows v - 128 + centred squared norms |v'|^2.  The
//                distance is shift-invariant: |q - t|^2 = |q'|^2 + |t'|^2 - 2 q'.t'.
//  k_bf_i8       block = 4 waves x 32 queries; 128-row train tiles double-buffered in LDS,
//                prefetched one tile ahead with buffer loads; per 32-row sub-tile each wave runs
//                4 MFMAs (train rows = A, its queries = B), the next sub-tile's MFMAs issued
//                before this one's epilogue.  Each lane owns one query and 16 train rows; it
//                forms keys 16 s + (15 - reg) with s = 2 q'.t' - |t'|^2 = |q'|^2 - d^2 (one
//                v_lshl_add per candidate, the norm term staged in LDS), takes the sub-tile's
//                two largest keys (v_med3 / v_max chains) and inserts them into its running
//                top-2: the (distance, index) order OpenCV's knnMatch produces.
// Cross-check path, bf16 (VO_BF_BF16=1, identical results):
//  k_bf_prep / k_bf_mfma  bf16 rows, 9 v_mfma_f32_32x32x16_bf16 per sub-tile (the ninth K-step
//                folds |t|^2 in), running top-2 of s with strict '>' in increasing train index.
// Both:
//  k_bf_merge  merges the train splits (grid filling for small batches) and writes
//              idx2 / dist2 = sqrtf(d2) (correctly rounded, as OpenCV's sqrt).
//  k_bf_fixup  integer order equals float order only while sqrtf separates the integers
//              involved: below 2^22 it always does.  A query whose second distance^2 reaches
//              2^22 (impossible for real SIFT descriptors, whose norms are ~512) is recomputed
//              exactly in float order by this slow path.
#include "vo_dev.h"

#include <float.h>
#include <limits.h>

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

#define BF_QB 128          // queries per block
#define BF_TT 64           // train rows per LDS tile (bf16 kernel)
#define BFI_TT 128         // train rows per LDS tile (int8 kernel; measured: 64 rows 12 % slower)
#define BF_MAXSPLIT 16
#define BF_SAFE (1 << 22)  // below this, distinct integer d2 have distinct sqrtf

struct BfArgs {
    int B, qcap, tcap, tsplit;
    int tt;                // train rows per tile of the launched kernel (splits are multiples)
    int qb;                // queries per block
    const __bf16* qbf;     // [B][qcap][128]
    const __bf16* tbf;     // [B][tcap][128]
    const int32_t* qn;     // [B][qcap] |q|^2
    const int32_t* tn;     // [B][tcap] |t|^2
    const int32_t* nq;     // [B]
    const int32_t* nt;     // [B]
    int4* part;            // [B][tsplit][qcap] (d0', i0, d1', i1) per split
    int32_t* idx2;         // [B][qcap][2]
    float* dist2;          // [B][qcap][2]
    int32_t* flag_n;       // fixup list length
    int32_t* flag_list;    // [B * qcap] b * qcap + q
    // device work plan (int8 path, B <= BF_PLAN_MAXB): the splits come from the device counts, not
    // the capacities, and the kernel's blocks loop over the (problem, query block, split) items
    int planned;
    int32_t* plan;         // [B + 2]: item prefix per problem, then the common split count
};

#define BF_PLAN_MAXB 1024   // problems the device plan handles (larger batches: capacity plan)
#define BF_TARGET 2048      // work items the plan aims at (8 per CU)

// Per-problem split of the planned path: nqb query blocks, sp train splits of `per` rows (a
// multiple of the tile rows), from the counts and the batch-wide split count sp_all.
struct BfPlan {
    int nqb, sp, per;
};
VO_DEV BfPlan bf_plan(int nq, int nt, int sp_all, int tt)
{
    BfPlan p;
    p.nqb = nq > 0 ? (nq + BF_QB - 1) / BF_QB : 0;
    const int tiles = (nt + tt - 1) / tt;
    p.sp = max(1, min(sp_all, tiles));
    p.per = (((nt + p.sp - 1) / p.sp + tt - 1) / tt) * tt;
    return p;
}

// train rows per split of a problem with nt rows (a multiple of the tile rows)
VO_DEV int bf_per(int nt, const BfArgs& A) { return (((nt + A.tsplit - 1) / A.tsplit) + A.tt - 1) / A.tt * A.tt; }

// (d, i) lexicographic order; absent entries are (INT_MAX, -1) and never precede a real one
VO_DEV bool lex_lt(int da, int ia, int db, int ib) { return da < db || (da == db && (unsigned)ia < (unsigned)ib); }

VO_DEV void merge2(int& d0, int& i0, int& d1, int& i1, int e0, int j0, int e1, int j1)
{
    int r0, s0, r1, s1;
    if (lex_lt(d0, i0, e0, j0)) {
        r0 = d0; s0 = i0;
        if (lex_lt(d1, i1, e0, j0)) { r1 = d1; s1 = i1; } else { r1 = e0; s1 = j0; }
    } else {
        r0 = e0; s0 = j0;
        if (lex_lt(e1, j1, d0, i0)) { r1 = e1; s1 = j1; } else { r1 = d0; s1 = i0; }
    }
    d0 = r0; i0 = s0; d1 = r1; i1 = s1;
}

// descriptors -> bf16 (times `mul`: 2 for queries, 1 for train rows; exact for integers
// 0..255) + |v|^2; rows >= n untouched (never read)
__global__ void __launch_bounds__(256) k_bf_prep(const float* __restrict__ src, const int32_t* n, int B, int cap,
                                                 float mul, __bf16* __restrict__ dst, int32_t* __restrict__ nrm)
{
    const int row = blockIdx.x * 4 + wave_id();
    const int b = row / cap, r = row - b * cap;
    if (b >= B || r >= n[b]) return;
    const int lane = lane_id();
    const float2 v = *reinterpret_cast<const float2*>(src + (int64_t)row * 128 + 2 * lane);
    const int a = (int)v.x, c = (int)v.y;
    __bf16* o = dst + (int64_t)row * 128 + 2 * lane;
    o[0] = (__bf16)(v.x * mul);
    o[1] = (__bf16)(v.y * mul);
    const int s = wave_sum_dpp(a * a + c * c);
    if (lane == 0) nrm[row] = s;
}

// The |t|^2 term rides in the MFMA as a ninth K-step: train row t carries its norm split into
// bytes (tn = a * 65536 + b * 256 + c) in K columns 128..130 and every query carries
// (-65536, -256, -1) there, while the queries' descriptor columns hold 2q.  The accumulator is
// then exactly s = 2 q.t - |t|^2 = |q|^2 - d^2 (every partial sum is an integer below 2^24),
// and the top-2 is a running maximum of s.  Absent train rows carry a = 255 (s < -2^24 + ...),
// below BF_FLOOR, which no real row reaches (s >= -|t|^2 >= -128 * 255^2).
#define BF_FLOOR (-16500000.f)
__global__ void __launch_bounds__(256) k_bf_mfma(BfArgs A)
{
    __shared__ uint4 tile[2][BF_TT * 16];
    __shared__ uint4 tnp[2][BF_TT * 2];          // norm bytes (k = 128..135) | zeros (136..143)
    const int nqb = (A.qcap + A.qb - 1) / A.qb;
    int blk = blockIdx.x;
    const int sp = blk % A.tsplit;
    blk /= A.tsplit;
    const int qb = blk % nqb, b = blk / nqb;
    if (b >= A.B) return;
    const int nq = A.nq[b], nt = A.nt[b];
    const int q0 = qb * A.qb;
    if (q0 >= nq) return;
    const int per = bf_per(nt, A);
    const int tlo = sp * per, thi = min(nt, tlo + per);
    const int ntile = thi > tlo ? (thi - tlo + BF_TT - 1) / BF_TT : 0;
    const int tid = threadIdx.x, w = wave_id(), lane = lane_id();
    const int h = lane >> 5, col = lane & 31;
    const int qi = q0 + 32 * w + col;
    const bool qv = qi < nq;
    bf16x8 qf[8];
    {
        const __bf16* qrow = A.qbf + ((int64_t)b * A.qcap + (qv ? qi : q0)) * 128 + 8 * h;
#pragma unroll
        for (int s = 0; s < 8; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(qrow + 16 * s);
    }
    bf16x8 qn9 = {};                              // K columns 128..135 / 136..143 of every query
    if (h == 0) { qn9[0] = (__bf16)(-65536.f); qn9[1] = (__bf16)(-256.f); qn9[2] = (__bf16)(-1.f); }
    const uint4* Tg = reinterpret_cast<const uint4*>(A.tbf + (int64_t)b * A.tcap * 128);
    const int32_t* TN = A.tn + (int64_t)b * A.tcap;
    uint4 pre[4];
    int pren = 255 << 16;
    auto gload = [&](int t0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int g = tid + 256 * i, row = g >> 4, slot = g & 15;
            const int r = t0 + row;
            pre[i] = r < thi ? Tg[(int64_t)r * 16 + slot] : make_uint4(0u, 0u, 0u, 0u);
        }
        pren = (tid < BF_TT && t0 + tid < thi) ? TN[t0 + tid] : (255 << 16);
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int g = tid + 256 * i, row = g >> 4, slot = g & 15;
            tile[buf][row * 16 + (slot ^ (row & 15))] = pre[i];
        }
        if (tid < BF_TT) {
            bf16x8 nb = {};
            nb[0] = (__bf16)(float)(pren >> 16);
            nb[1] = (__bf16)(float)((pren >> 8) & 255);
            nb[2] = (__bf16)(float)(pren & 255);
            tnp[buf][2 * tid] = *reinterpret_cast<const uint4*>(&nb);
            tnp[buf][2 * tid + 1] = make_uint4(0u, 0u, 0u, 0u);
        }
    };
    float s0 = BF_FLOOR, s1 = BF_FLOOR;
    int i0 = -1, i1 = -1;
    if (ntile > 0) {
        gload(tlo);
        lstore(0);
    }
    __syncthreads();
    for (int k = 0; k < ntile; ++k) {
        const int buf = k & 1, t0 = tlo + BF_TT * k;
        if (k + 1 < ntile) gload(t0 + BF_TT);          // next tile in flight during the MFMAs
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
            const int row = sub * 32 + col;
            f32x16 acc = {};
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                const bf16x8 af = *reinterpret_cast<const bf16x8*>(&tile[buf][row * 16 + ((2 * s + h) ^ (row & 15))]);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, qf[s], acc, 0, 0, 0);
            }
            {
                const bf16x8 af = *reinterpret_cast<const bf16x8*>(&tnp[buf][2 * row + h]);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, qn9, acc, 0, 0, 0);
            }
            // C layout: column = lane & 31 (query), row = (reg & 3) + 8 * (reg >> 2) + 4 * h (train)
            float m = acc[0];
#pragma unroll
            for (int reg = 1; reg < 16; ++reg) m = fmaxf(m, acc[reg]);
            if (m > s1) {
                const int ib = t0 + sub * 32 + 4 * h;
#pragma unroll
                for (int reg = 0; reg < 16; ++reg) {
                    const float v = acc[reg];
                    if (v > s1) {                       // rare: lanes whose candidate enters
                        const int ix = ib + (reg & 3) + 8 * (reg >> 2);
                        const bool c0 = v > s0;
                        s1 = c0 ? s0 : v;
                        i1 = c0 ? i0 : ix;
                        s0 = c0 ? v : s0;
                        i0 = c0 ? ix : i0;
                    }
                }
            }
        }
        if (k + 1 < ntile) lstore(buf ^ 1);
        __syncthreads();
    }
    // d' = |t|^2 - 2 q.t = -s (absent: INT_MAX); the two half-waves hold the same queries
    int d0 = i0 >= 0 ? -(int)s0 : INT_MAX, d1 = i1 >= 0 ? -(int)s1 : INT_MAX;
    merge2(d0, i0, d1, i1, __shfl_xor(d0, 32, 64), __shfl_xor(i0, 32, 64), __shfl_xor(d1, 32, 64),
           __shfl_xor(i1, 32, 64));
    if (h == 0 && qv) A.part[((int64_t)b * A.tsplit + sp) * A.qcap + qi] = make_int4(d0, i0, d1, i1);
}

// ---- i8 path (default).  Descriptors are integers 0..255, so v - 128 is an exact int8 and
// |q - t|^2 = |q'|^2 + |t'|^2 - 2 q'.t' with q' = q - 128, t' = t - 128 (the distance is
// shift-invariant); v_mfma_i32_32x32x32_i8 forms q'.t' exactly in int32 at twice the bf16 rate.
// The lane keeps the running top-2 of s = 2 q'.t' - |t'|^2 (= |q'|^2 - d^2), as k_bf_mfma does.
// (cv2compat.knnMatch rejects values outside 0..255, which would wrap in the int8 encoding.)
//
//  k_bf_prep_i8  descriptors -> int8 rows (v - 128) + centred squared norms |v'|^2; eight
//                threads per row, 16 values each (four float4 loads, one 16-byte store)
//  k_bf_i8       block = 4 waves x 32 queries; TT = 128-row int8 train tiles double-buffered in
//                LDS (16-B slots swizzled by (row >> 1) & 7), the next tile prefetched by buffer
//                loads during the MFMAs.  Per 32-row sub-tile a wave runs 4 MFMAs (one per
//                32-byte K chunk) with the train rows as A and its queries as B; the next
//                sub-tile's MFMAs are issued before this one's epilogue.  Lane (r, g) supplies
//                bytes 16g..16g+15 of every 32-byte K chunk for both operands: the same k for the
//                same (g, element) on both sides, so the MFMA sums every k of the chunk once
//                whatever the hardware's k order inside a chunk.
//                Epilogue: key = (acc << 5) + 16 (-|t'|^2) + (15 - reg) = 16 s + (15 - reg) per
//                accumulator register (the staged ntn row term), so the largest key is the
//                largest s with ties to the lowest train index of the lane; the sub-tile's two
//                largest keys come from four v_max / v_med3 running top-2 chains merged pairwise,
//                and only they are tested against the lane's running second-best.
// Both operands in one launch: blocks [0, qblocks) prepare the queries, the rest the train rows;
// block 0 also clears the fixup-list counter (the merge appends to it later in stream order).
struct BfPrep {
    const float* src;
    const int32_t* n;
    int cap;
    int8_t* dst;
    int32_t* nrm;
};
__global__ void __launch_bounds__(256) k_bf_prep_i8(BfPrep Q, BfPrep T, int B, int qblocks, int32_t* flag_n)
{
    if (blockIdx.x == 0 && threadIdx.x == 0) *flag_n = 0;
    // grid-stride over the 32-row groups of both operands (queries first); a group past its
    // problem's count is skipped with one load, so the grid need not cover the capacities
    const int64_t gq = (int64_t)B * ((Q.cap + 31) / 32), gt = (int64_t)B * ((T.cap + 31) / 32);
    (void)qblocks;
    for (int64_t g = blockIdx.x; g < gq + gt; g += gridDim.x) {
        const bool isq = g < gq;
        const BfPrep& X = isq ? Q : T;
        const int gpc = (X.cap + 31) / 32;
        const int64_t gg = isq ? g : g - gq;
        const int b = (int)(gg / gpc), r = (int)(gg - (int64_t)b * gpc) * 32 + (threadIdx.x >> 3), part = threadIdx.x & 7;
        const int nb = X.n[b];
        if ((int)(gg - (int64_t)b * gpc) * 32 >= nb) continue;           // block-uniform
        const bool ok = r < nb && r < X.cap;
        const int64_t row = (int64_t)b * X.cap + r;
        int ss = 0;
        if (ok) {
            const float4* s4 = reinterpret_cast<const float4*>(X.src + row * 128 + 16 * part);
            uint32_t w[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float4 v = s4[k];
                const int a0 = (int)v.x - 128, a1 = (int)v.y - 128, a2 = (int)v.z - 128, a3 = (int)v.w - 128;
                ss += a0 * a0 + a1 * a1 + a2 * a2 + a3 * a3;
                w[k] = (uint32_t)(a0 & 255) | ((uint32_t)(a1 & 255) << 8) | ((uint32_t)(a2 & 255) << 16) |
                       ((uint32_t)(a3 & 255) << 24);
            }
            *reinterpret_cast<uint4*>(X.dst + row * 128 + 16 * part) = make_uint4(w[0], w[1], w[2], w[3]);
        }
        ss += __shfl_xor(ss, 1, 64);
        ss += __shfl_xor(ss, 2, 64);
        ss += __shfl_xor(ss, 4, 64);
        if (ok && part == 0) X.nrm[row] = ss;
    }
}

// middle of three (v_med3_i32): with hi >= lo, med3(hi, lo, v) = max(lo, min(hi, v))
VO_DEV int med3_i32(int a, int b, int c)
{
    int r;
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
#define BFI_FLOOR (-(1 << 25))      // below every real s = 2 q'.t' - |t'|^2 >= -3 * 2^21
#define BFI_ABSENT_KEY (-(1 << 30)) // staged key term of absent train rows: s <= -2^26 < BFI_FLOOR

// TT train rows per LDS tile, QG groups of 32 queries per wave (a train fragment read from LDS
// feeds QG MFMAs; QG = 2 measured 30 % slower: 150 VGPRs, 3 waves per SIMD).  The vector unit,
// not the matrix pipe, bounds this kernel: ~3 VALU instructions per (query, train) candidate
// (key, v_med3, v_max) against 1/8 MFMA cycle.
template <int TT, int QG>
__global__ void __launch_bounds__(256) k_bf_i8(BfArgs A)
{
    static_assert(TT % 32 == 0 && TT <= 256, "tile rows");
    constexpr int NPRE = TT * 8 / 256;            // 16-byte slots per thread per tile
    __shared__ uint4 tile[2][TT * 8];             // TT rows x 128 B
    __shared__ int ntn[2][TT];                    // -|t'|^2 per row
    __shared__ int pref_s[BF_PLAN_MAXB + 1];      // planned path: work items before problem b
    __shared__ int scan_s[16];
    const int tid = threadIdx.x, w = wave_id(), lane = lane_id();
    // Work items.  Planned (A.planned): every block derives the same plan from the device counts
    // -- query blocks per problem, one split count sp_all for the batch that brings the items to
    // about BF_TARGET, items (problem, query block, split) in that order -- and the blocks loop
    // over the items; block 0 publishes the item prefix for the merge.  Otherwise one item per
    // block from the capacities (blockIdx -> split, query block, problem).
    int total = gridDim.x, sp_all = 1;
    if (A.planned) {
        const int B = A.B, per_t = (B + 255) / 256, lo = min(B, tid * per_t), hi = min(B, lo + per_t);
        int my_qb = 0;
        for (int b = lo; b < hi; ++b) my_qb += bf_plan(A.nq[b], A.nt[b], 1, TT).nqb;
        int tot_qb;
        block_scan_i32(my_qb, scan_s, &tot_qb);
        sp_all = tot_qb > 0 ? min(BF_MAXSPLIT, max(1, (BF_TARGET + tot_qb - 1) / tot_qb)) : 1;
        int my_items = 0;
        for (int b = lo; b < hi; ++b) {
            const BfPlan p = bf_plan(A.nq[b], A.nt[b], sp_all, TT);
            my_items += p.nqb * p.sp;
        }
        int run = block_scan_i32(my_items, scan_s, &total);
        for (int b = lo; b < hi; ++b) {
            pref_s[b] = run;
            const BfPlan p = bf_plan(A.nq[b], A.nt[b], sp_all, TT);
            run += p.nqb * p.sp;
        }
        if (tid == 0) pref_s[B] = total;
        __syncthreads();
        if (blockIdx.x == 0) {
            for (int b = tid; b <= B; b += 256) A.plan[b] = pref_s[b];
            if (tid == 0) A.plan[B + 1] = sp_all;
        }
    }
    for (int item = blockIdx.x; item < total; item += gridDim.x) {      // block-uniform loop
    int b, qb, sp, per;
    int64_t prow;                                 // partial-result row of query q0 of this item
    if (A.planned) {
        int l = 0, h = A.B;                       // pref_s[l] <= item < pref_s[l + 1]
        while (h - l > 1) {
            const int m = (l + h) >> 1;
            if (pref_s[m] <= item) l = m; else h = m;
        }
        b = l;
        const BfPlan p = bf_plan(A.nq[b], A.nt[b], sp_all, TT);
        const int local = item - pref_s[b];
        qb = local / p.sp;
        sp = local - qb * p.sp;
        per = p.per;
        prow = (int64_t)item * BF_QB;
    } else {
        const int nqb = (A.qcap + A.qb - 1) / A.qb;
        int blk = item;
        sp = blk % A.tsplit;
        blk /= A.tsplit;
        qb = blk % nqb;
        b = blk / nqb;
        if (b >= A.B) continue;
        per = bf_per(A.nt[b], A);
        prow = ((int64_t)b * A.tsplit + sp) * A.qcap + (int64_t)qb * A.qb;
    }
    const int nq = A.nq[b], nt = A.nt[b];
    const int q0 = qb * A.qb;
    if (q0 >= nq) continue;
    const int tlo = sp * per, thi = min(nt, tlo + per);
    const int ntile = thi > tlo ? (thi - tlo + TT - 1) / TT : 0;
    const int h = lane >> 5, col = lane & 31;
    const int8_t* qi8 = reinterpret_cast<const int8_t*>(A.qbf);
    v4i qf[QG][4];
#pragma unroll
    for (int g = 0; g < QG; ++g) {
        const int qi = q0 + 32 * (QG * w + g) + col;
        const int8_t* qrow = qi8 + ((int64_t)b * A.qcap + (qi < nq ? qi : q0)) * 128 + 16 * h;
#pragma unroll
        for (int c = 0; c < 4; ++c) qf[g][c] = *reinterpret_cast<const v4i*>(qrow + 32 * c);
    }
    // the split's rows through buffer resources sized to end at thi: rows past it read as
    // zero (no per-row branch, so the prefetch stays in flight across the MFMAs)
    const int8_t* Tb = reinterpret_cast<const int8_t*>(A.tbf) + ((int64_t)b * A.tcap + tlo) * 128;
    const int32_t* TN = A.tn + (int64_t)b * A.tcap;
    const __amdgpu_buffer_rsrc_t rT = __builtin_amdgcn_make_buffer_rsrc((void*)Tb, (short)0, (thi - tlo) * 128, 0x00020000);
    const __amdgpu_buffer_rsrc_t rN =
        __builtin_amdgcn_make_buffer_rsrc((void*)(TN + tlo), (short)0, (thi - tlo) * 4, 0x00020000);
    v4i pre[NPRE];
    int pren = 0;
    // loop-invariant per-lane offsets, tile offset in the scalar offset: no address VGPR that the
    // MFMA results could be allocated over while a load is in flight
    const int vT = tid * 16, vN = (tid & (TT - 1)) * 4;
    auto gload = [&](int t0) {
#pragma unroll
        for (int i = 0; i < NPRE; ++i)
            pre[i] = __builtin_amdgcn_raw_buffer_load_b128(rT, vT, (t0 - tlo) * 128 + 4096 * i, 0);
        pren = __builtin_amdgcn_raw_buffer_load_b32(rN, vN, (t0 - tlo) * 4, 0);
    };
    // 16-byte slot j of row r lives at slot j ^ ((r >> 1) & 7): the 16 rows of a ds_read_b128
    // lane group ({0-3,12-15,20-27} / {4-11,16-19,28-31}) then cover all 64 banks once
    auto lstore = [&](int buf, int t0) {
#pragma unroll
        for (int i = 0; i < NPRE; ++i) {
            const int e = tid + 256 * i, row = e >> 3, slot = e & 7;
            tile[buf][row * 8 + (slot ^ ((row >> 1) & 7))] = make_uint4(pre[i].x, pre[i].y, pre[i].z, pre[i].w);
        }
        if (tid < TT) {
            // key term of row tid: 16 (-|t'|^2) + (15 - reg), reg = the accumulator register that
            // holds this row in the 32x32 C layout (row bits 0-1 = reg & 3, bits 3-4 = reg >> 2)
            const int rl = tid & 31, reg = (rl & 3) | ((rl >> 3) << 2);
            ntn[buf][tid] = t0 + tid < thi ? (-pren) * 16 + (15 - reg) : BFI_ABSENT_KEY;
        }
    };
    int s0[QG], s1[QG], i0[QG], i1[QG], thr[QG];      // thr = 16 s1 + 15: key > thr <=> s > s1
#pragma unroll
    for (int g = 0; g < QG; ++g) { s0[g] = s1[g] = BFI_FLOOR; i0[g] = i1[g] = -1; thr[g] = 16 * BFI_FLOOR + 15; }
    if (ntile > 0) {
        gload(tlo);
        lstore(0, tlo);
    }
    // every load so far complete on every path: otherwise the loop inherits "query fragments
    // may be pending" from the ntile == 0 path and waits on the prefetch before each MFMA
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    for (int k = 0; k < ntile; ++k) {
        const int buf = k & 1, t0 = tlo + TT * k;
        if (k + 1 < ntile) gload(t0 + TT);             // next tile in flight during the MFMAs
        auto mfma_sub = [&](int sub, v16i* acc) {
            const int row = sub * 32 + col;
#pragma unroll
            for (int g = 0; g < QG; ++g) acc[g] = v16i{};
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const uint4 u = tile[buf][row * 8 + ((2 * c + h) ^ ((row >> 1) & 7))];
                const v4i af = {(int)u.x, (int)u.y, (int)u.z, (int)u.w};
#pragma unroll
                for (int g = 0; g < QG; ++g)
                    acc[g] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af, qf[g][c], acc[g], 0, 0, 0);
            }
        };
        auto epilogue = [&](int sub, v16i* acc) {
            // C layout: column = lane & 31 (query), row = (reg & 3) + 8 * (reg >> 2) + 4 * h (train).
            // key = 32 q'.t' + 16 (-|t'|^2) + (15 - reg) = 16 s + (15 - reg): the largest key is the
            // largest s, ties to the lowest register = the lowest train index of the lane
            const int4* n4 = reinterpret_cast<const int4*>(&ntn[buf][sub * 32 + 4 * h]);
            int4 nv[4];
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) nv[g4] = n4[2 * g4];     // rows 8 g4 + 4h + 0..3
            const int rbase = t0 + sub * 32 + 4 * h;
#pragma unroll
            for (int g = 0; g < QG; ++g) {
                int kk[16];
#pragma unroll
                for (int g4 = 0; g4 < 4; ++g4) {
                    kk[4 * g4 + 0] = (acc[g][4 * g4 + 0] << 5) + nv[g4].x;
                    kk[4 * g4 + 1] = (acc[g][4 * g4 + 1] << 5) + nv[g4].y;
                    kk[4 * g4 + 2] = (acc[g][4 * g4 + 2] << 5) + nv[g4].z;
                    kk[4 * g4 + 3] = (acc[g][4 * g4 + 3] << 5) + nv[g4].w;
                }
                // the lane's two largest keys of the sub-tile (only they can enter its top-2; keys
                // are distinct in the low bits): four running top-2 chains (v_med3 + v_max per
                // key), merged pairwise (hi = max, lo = med3(a1, b1, max(a2, b2)))
                int t1[4], t2[4];
#pragma unroll
                for (int q4 = 0; q4 < 4; ++q4) {
                    const int* v = kk + 4 * q4;
                    t1[q4] = max(v[0], v[1]);
                    t2[q4] = min(v[0], v[1]);
                    t2[q4] = med3_i32(t1[q4], t2[q4], v[2]);
                    t1[q4] = max(t1[q4], v[2]);
                    t2[q4] = med3_i32(t1[q4], t2[q4], v[3]);
                    t1[q4] = max(t1[q4], v[3]);
                }
                const int u1 = max(t1[0], t1[1]), u2 = med3_i32(t1[0], t1[1], max(t2[0], t2[1]));
                const int w1 = max(t1[2], t1[3]), w2 = med3_i32(t1[2], t1[3], max(t2[2], t2[3]));
                const int m = max(u1, w1), m2 = med3_i32(u1, w1, max(u2, w2));
                auto insert = [&](int key) {
                    const int sv = key >> 4, reg = 15 - (key & 15);
                    const int ix = rbase + (reg & 3) + 8 * (reg >> 2);
                    const bool in = key > thr[g], c0 = sv > s0[g];
                    s1[g] = in ? (c0 ? s0[g] : sv) : s1[g];
                    i1[g] = in ? (c0 ? i0[g] : ix) : i1[g];
                    s0[g] = in && c0 ? sv : s0[g];
                    i0[g] = in && c0 ? ix : i0[g];
                    thr[g] = 16 * s1[g] + 15;
                };
                insert(m);
                if (__builtin_expect(m2 > thr[g], 0)) insert(m2);     // both entered somewhere in the wave
            }
        };
        // software pipeline: the next sub-tile's MFMAs are issued before this one's epilogue, so
        // the matrix pipe works while the vector unit forms keys and the top-2
        v16i accA[QG], accB[QG];
        mfma_sub(0, accA);
#pragma unroll
        for (int sub = 0; sub < TT / 32; ++sub) {
            v16i* cur = (sub & 1) ? accB : accA;
            v16i* nxt = (sub & 1) ? accA : accB;
            if (sub + 1 < TT / 32) mfma_sub(sub + 1, nxt);
            epilogue(sub, cur);
        }
        if (k + 1 < ntile) lstore(buf ^ 1, t0 + TT);
        __syncthreads();
    }
    // d' = |t'|^2 - 2 q'.t' = -s (absent: INT_MAX); the two half-waves hold the same queries
#pragma unroll
    for (int g = 0; g < QG; ++g) {
        const int qi = q0 + 32 * (QG * w + g) + col;
        int d0 = i0[g] >= 0 ? -s0[g] : INT_MAX, d1 = i1[g] >= 0 ? -s1[g] : INT_MAX;
        int j0 = i0[g], j1 = i1[g];
        merge2(d0, j0, d1, j1, __shfl_xor(d0, 32, 64), __shfl_xor(j0, 32, 64), __shfl_xor(d1, 32, 64),
               __shfl_xor(j1, 32, 64));
        if (h == 0 && qi < nq) A.part[prow + (qi - q0)] = make_int4(d0, j0, d1, j1);
    }
    __syncthreads();                              // the next item restages the LDS tiles
    }                                             // items
}

__global__ void __launch_bounds__(256) k_bf_merge(BfArgs A)
{
    const int row = blockIdx.x * blockDim.x + threadIdx.x;
    const int b = row / A.qcap, q = row - b * A.qcap;
    if (b >= A.B) return;
    if (q >= A.nq[b]) {                      // no query: the absent pair (-1, FLT_MAX) x 2
        int32_t* ix = A.idx2 + ((int64_t)b * A.qcap + q) * 2;
        float* ds = A.dist2 + ((int64_t)b * A.qcap + q) * 2;
        ix[0] = ix[1] = -1;
        ds[0] = ds[1] = FLT_MAX;
        return;
    }
    int d0 = INT_MAX, d1 = INT_MAX, i0 = -1, i1 = -1;
    if (A.planned) {
        // the items of (b, q's query block) are consecutive, one per split (k_bf_i8's plan)
        const BfPlan p = bf_plan(A.nq[b], A.nt[b], A.plan[A.B + 1], A.tt);
        const int qb = q / BF_QB;
        const int64_t it0 = A.plan[b] + (int64_t)qb * p.sp;
        for (int sp = 0; sp < p.sp; ++sp) {
            const int4 v = A.part[(it0 + sp) * BF_QB + (q - qb * BF_QB)];
            merge2(d0, i0, d1, i1, v.x, v.y, v.z, v.w);
        }
    } else {
        const int per = bf_per(A.nt[b], A);
        for (int sp = 0; sp < A.tsplit; ++sp) {
            if (sp * per >= A.nt[b]) break;            // empty split: its block never ran
            const int4 p = A.part[((int64_t)b * A.tsplit + sp) * A.qcap + q];
            merge2(d0, i0, d1, i1, p.x, p.y, p.z, p.w);
        }
    }
    const int qn = A.qn[(int64_t)b * A.qcap + q];
    int32_t* ix = A.idx2 + ((int64_t)b * A.qcap + q) * 2;
    float* ds = A.dist2 + ((int64_t)b * A.qcap + q) * 2;
    const int e0 = i0 >= 0 ? d0 + qn : 0, e1 = i1 >= 0 ? d1 + qn : 0;
    ix[0] = i0;
    ix[1] = i1;
    ds[0] = i0 >= 0 ? sqrtf((float)e0) : FLT_MAX;
    ds[1] = i1 >= 0 ? sqrtf((float)e1) : FLT_MAX;
    if (e0 >= BF_SAFE || e1 >= BF_SAFE) A.flag_list[atomicAdd(A.flag_n, 1)] = row;
}

// exact float-order 2-NN for the flagged queries (one wave per query, fp32 inputs)
__global__ void __launch_bounds__(256) k_bf_fixup(BfArgs A, const float* __restrict__ q, const float* __restrict__ t)
{
    const int nflag = *A.flag_n;
    const int lane = lane_id();
    for (int f = blockIdx.x * 4 + wave_id(); f < nflag; f += gridDim.x * 4) {
        const int row = A.flag_list[f];
        const int b = row / A.qcap, qi = row - b * A.qcap;
        const int nt = A.nt[b];
        const float* qr = q + (int64_t)row * 128;
        float e0 = FLT_MAX, e1 = FLT_MAX;
        int j0 = -1, j1 = -1;
        for (int j = lane; j < nt; j += 64) {       // each lane: rows lane, lane + 64, ... in order
            const float* tr = t + ((int64_t)b * A.tcap + j) * 128;
            int d2 = 0;
            for (int k = 0; k < 128; ++k) {
                const int dd = (int)qr[k] - (int)tr[k];
                d2 += dd * dd;
            }
            const float d = sqrtf((float)d2);
            if (d < e1) {
                if (d < e0) { e1 = e0; j1 = j0; e0 = d; j0 = j; }
                else { e1 = d; j1 = j; }
            }
        }
        // lane merge in (distance, index) order
        for (int o = 1; o < 64; o <<= 1) {
            const float f0 = __shfl_xor(e0, o, 64), f1 = __shfl_xor(e1, o, 64);
            const int k0 = __shfl_xor(j0, o, 64), k1 = __shfl_xor(j1, o, 64);
            auto lt = [](float da, int ia, float db, int ib) { return da < db || (da == db && (unsigned)ia < (unsigned)ib); };
            float r0, r1;
            int s0, s1;
            if (lt(e0, j0, f0, k0)) { r0 = e0; s0 = j0; if (lt(e1, j1, f0, k0)) { r1 = e1; s1 = j1; } else { r1 = f0; s1 = k0; } }
            else { r0 = f0; s0 = k0; if (lt(f1, k1, e0, j0)) { r1 = f1; s1 = k1; } else { r1 = e0; s1 = j0; } }
            e0 = r0; j0 = s0; e1 = r1; j1 = s1;
        }
        if (lane == 0) {
            int32_t* ix = A.idx2 + ((int64_t)b * A.qcap + qi) * 2;
            float* ds = A.dist2 + ((int64_t)b * A.qcap + qi) * 2;
            ix[0] = j0; ix[1] = j1;
            ds[0] = e0; ds[1] = e1;
        }
    }
}

}  // namespace

// ======================================================================= host side
#define VO_STREAM(s) ((hipStream_t)(s))

static int bf_tsplit(int B, int qcap, int tcap, int qb, int tt)
{
    const int blocks = B * ((qcap + qb - 1) / qb);
    int sp = (2048 + blocks - 1) / blocks;              // about 8 blocks per CU
    const int tiles = (tcap + tt - 1) / tt;
    if (sp > tiles) sp = tiles;
    if (sp > BF_MAXSPLIT) sp = BF_MAXSPLIT;
    return sp < 1 ? 1 : sp;
}

// the most splits any kernel configuration below uses (sizes the partial-result scratch)
static int bf_tsplit_max(int B, int qcap, int tcap) { return bf_tsplit(B, qcap, tcap, BF_QB, BF_TT); }

static int64_t align256(int64_t v) { return (v + 255) & ~(int64_t)255; }

// partial-result rows: the capacity plan's [B][tsplit][qcap], or the device plan's items x 128
// (items <= max(B x query blocks, 2 x BF_TARGET): one split when the query blocks alone reach the
// target, otherwise at most target + query blocks)
static int64_t bf_part_rows(int B, int qcap, int tcap)
{
    const int64_t cap_rows = (int64_t)B * bf_tsplit_max(B, qcap, tcap) * qcap;
    const int64_t nqb = (qcap + BF_QB - 1) / BF_QB;
    const int64_t items = (int64_t)B * nqb > 2 * BF_TARGET ? (int64_t)B * nqb : 2 * BF_TARGET;
    return cap_rows > items * BF_QB ? cap_rows : items * BF_QB;
}

extern "C" int64_t vo_bf_knn2_batch_scratch(int B, int32_t qcap, int32_t tcap)
{
    if (B < 1 || qcap < 1 || tcap < 1) return -1;
    return align256((int64_t)B * qcap * 256) + align256((int64_t)B * tcap * 256) + align256((int64_t)B * qcap * 4) +
           align256((int64_t)B * tcap * 4) + align256(bf_part_rows(B, qcap, tcap) * 16) + 256 +
           align256((int64_t)B * qcap * 4) + align256((int64_t)(B + 2) * 4);
}

extern "C" int vo_bf_knn2_batch(int B, const float* q, const int32_t* nq, int32_t qcap, const float* t,
                                const int32_t* nt, int32_t tcap, int32_t dim, int32_t* idx2, float* dist2,
                                void* scratch, int64_t scratch_bytes, vo_stream_t stream)
{
    if (B < 1 || !q || !nq || !t || !nt || !idx2 || !dist2 || !scratch || dim != 128 || qcap < 1 || tcap < 1)
        return VO_EARG;
    if (scratch_bytes < vo_bf_knn2_batch_scratch(B, qcap, tcap)) return VO_EARG;
    hipStream_t st = VO_STREAM(stream);
    BfArgs A;
    // int8 MFMA path unless VO_BF_BF16=1 (the bf16 path; identical results, kept as its cross-check)
    const char* bf16_env = getenv("VO_BF_BF16");
    const bool use_bf16 = bf16_env && bf16_env[0] == '1';
    const int tt = use_bf16 ? BF_TT : BFI_TT;
    A.B = B; A.qcap = qcap; A.tcap = tcap; A.qb = BF_QB; A.tsplit = bf_tsplit(B, qcap, tcap, A.qb, tt);
    A.tt = tt;
    char* p = (char*)scratch;
    A.qbf = (const __bf16*)p; p += align256((int64_t)B * qcap * 256);
    A.tbf = (const __bf16*)p; p += align256((int64_t)B * tcap * 256);
    A.qn = (const int32_t*)p; p += align256((int64_t)B * qcap * 4);
    A.tn = (const int32_t*)p; p += align256((int64_t)B * tcap * 4);
    A.part = (int4*)p; p += align256(bf_part_rows(B, qcap, tcap) * 16);
    A.flag_n = (int32_t*)p; p += 256;
    A.flag_list = (int32_t*)p; p += align256((int64_t)B * qcap * 4);
    A.plan = (int32_t*)p;
    A.nq = nq; A.nt = nt; A.idx2 = idx2; A.dist2 = dist2;
    const int nqb = (qcap + A.qb - 1) / A.qb;
    // int8 path: the device plan (splits from the real counts, not the capacities: a C3 call of 16
    // pairs of ~1,660 descriptors in 16,384-row buffers ran 208 blocks on 256 CUs with one split);
    // VO_BF_PLAN=0 keeps the capacity plan (A/B)
    const char* plan_e = getenv("VO_BF_PLAN");
    const int plan_env = plan_e ? atoi(plan_e) : 1;
    A.planned = !use_bf16 && plan_env != 0 && B <= BF_PLAN_MAXB;
    if (!use_bf16) {
        const int qblocks = (int)(((int64_t)B * qcap + 31) / 32), tblocks = (int)(((int64_t)B * tcap + 31) / 32);
        const BfPrep Q{q, nq, qcap, (int8_t*)A.qbf, (int32_t*)A.qn}, T{t, nt, tcap, (int8_t*)A.tbf, (int32_t*)A.tn};
        // grid-stride prep: up to 16 blocks per CU (groups past a problem's count are skipped)
        const int pblocks = qblocks + tblocks < 4096 ? qblocks + tblocks : 4096;
        hipLaunchKernelGGL(k_bf_prep_i8, dim3(pblocks), dim3(256), 0, st, Q, T, B, qblocks, A.flag_n);
        if (A.planned) hipLaunchKernelGGL((k_bf_i8<BFI_TT, 1>), dim3(BF_TARGET), dim3(256), 0, st, A);
        else hipLaunchKernelGGL((k_bf_i8<BFI_TT, 1>), dim3(B * nqb * A.tsplit), dim3(256), 0, st, A);
    } else {
        if (hipMemsetAsync(A.flag_n, 0, sizeof(int32_t), st) != hipSuccess) return VO_EHIP;
        hipLaunchKernelGGL(k_bf_prep, dim3(((int64_t)B * qcap + 3) / 4), dim3(256), 0, st, q, nq, B, qcap, 2.f,
                           (__bf16*)A.qbf, (int32_t*)A.qn);
        hipLaunchKernelGGL(k_bf_prep, dim3(((int64_t)B * tcap + 3) / 4), dim3(256), 0, st, t, nt, B, tcap, 1.f,
                           (__bf16*)A.tbf, (int32_t*)A.tn);
        hipLaunchKernelGGL(k_bf_mfma, dim3(B * nqb * A.tsplit), dim3(256), 0, st, A);
    }
    hipLaunchKernelGGL(k_bf_merge, dim3(((int64_t)B * qcap + 255) / 256), dim3(256), 0, st, A);
    hipLaunchKernelGGL(k_bf_fixup, dim3(64), dim3(256), 0, st, A, q, t);
    return hipGetLastError() == hipSuccess ? VO_OK : VO_EHIP;
}
