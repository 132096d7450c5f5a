// Batched brute-force 2-NN matcher on MFMA (cv2.BFMatcher().knnMatch(d0, d1, k=2),
// /root/reference/VisualOdometryPipeLine.py:36,229; SURVEY.md §8a row a4, §8d "BF kNN").
//
// B independent (query set, train set) problems per launch.  SIFT descriptors hold integers
// 0..255, so bf16 operands and fp32 accumulation are exact (sum <= 128 * 255^2 < 2^24) and
// the distances are those of OpenCV's float path bit for bit.
//
//  k_bf_prep   descriptors -> bf16 rows + integer squared norms (one wave per row)
//  k_bf_mfma   block = 4 waves x 32 queries; 64-row train tiles double-buffered in LDS (16-B
//              slots XOR-swizzled by row: conflict-free ds_read_b128); per 32-row sub-tile each
//              wave runs 9 v_mfma_f32_32x32x16_bf16 with the TRAIN rows as the A operand and its
//              queries as B, so every lane owns one query column and 16 train rows of the tile;
//              the ninth K-step folds |t|^2 in, so the accumulator is s = 2 q.t - |t|^2 exactly.
//              The lane keeps a running top-2 of s (= |q|^2 - d^2, |q|^2 constant per lane) with
//              strict '>' in increasing train index, i.e. the (distance, index) order OpenCV's
//              knnMatch produces; a per-lane max over the 16 candidates skips the insertion
//              when none can enter.
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
#define BF_TT 64           // train rows per LDS tile
#define BF_MAXSPLIT 16
#define BF_SAFE (1 << 22)  // below this, distinct integer d2 have distinct sqrtf

struct BfArgs {
    int B, qcap, tcap, tsplit;
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
};

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
    const int nqb = (A.qcap + BF_QB - 1) / BF_QB;
    int blk = blockIdx.x;
    const int sp = blk % A.tsplit;
    blk /= A.tsplit;
    const int qb = blk % nqb, b = blk / nqb;
    if (b >= A.B) return;
    const int nq = A.nq[b], nt = A.nt[b];
    const int q0 = qb * BF_QB;
    if (q0 >= nq) return;
    const int per = (((nt + A.tsplit - 1) / A.tsplit) + BF_TT - 1) & ~(BF_TT - 1);
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

__global__ void __launch_bounds__(256) k_bf_merge(BfArgs A)
{
    const int row = blockIdx.x * blockDim.x + threadIdx.x;
    const int b = row / A.qcap, q = row - b * A.qcap;
    if (b >= A.B || q >= A.nq[b]) return;
    int d0 = INT_MAX, d1 = INT_MAX, i0 = -1, i1 = -1;
    const int per = (((A.nt[b] + A.tsplit - 1) / A.tsplit) + BF_TT - 1) & ~(BF_TT - 1);
    for (int sp = 0; sp < A.tsplit; ++sp) {
        if (sp * per >= A.nt[b]) break;            // empty split: its block never ran
        const int4 p = A.part[((int64_t)b * A.tsplit + sp) * A.qcap + q];
        merge2(d0, i0, d1, i1, p.x, p.y, p.z, p.w);
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

static int bf_tsplit(int B, int qcap, int tcap)
{
    const int blocks = B * ((qcap + BF_QB - 1) / BF_QB);
    int sp = (2048 + blocks - 1) / blocks;              // about 8 blocks per CU
    const int tiles = (tcap + BF_TT - 1) / BF_TT;
    if (sp > tiles) sp = tiles;
    if (sp > BF_MAXSPLIT) sp = BF_MAXSPLIT;
    return sp < 1 ? 1 : sp;
}

static int64_t align256(int64_t v) { return (v + 255) & ~(int64_t)255; }

extern "C" int64_t vo_bf_knn2_batch_scratch(int B, int32_t qcap, int32_t tcap)
{
    if (B < 1 || qcap < 1 || tcap < 1) return -1;
    const int sp = bf_tsplit(B, qcap, tcap);
    return align256((int64_t)B * qcap * 256) + align256((int64_t)B * tcap * 256) + align256((int64_t)B * qcap * 4) +
           align256((int64_t)B * tcap * 4) + align256((int64_t)B * sp * qcap * 16) + 256 + align256((int64_t)B * qcap * 4);
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
    A.B = B; A.qcap = qcap; A.tcap = tcap; A.tsplit = bf_tsplit(B, qcap, tcap);
    char* p = (char*)scratch;
    A.qbf = (const __bf16*)p; p += align256((int64_t)B * qcap * 256);
    A.tbf = (const __bf16*)p; p += align256((int64_t)B * tcap * 256);
    A.qn = (const int32_t*)p; p += align256((int64_t)B * qcap * 4);
    A.tn = (const int32_t*)p; p += align256((int64_t)B * tcap * 4);
    A.part = (int4*)p; p += align256((int64_t)B * A.tsplit * qcap * 16);
    A.flag_n = (int32_t*)p; p += 256;
    A.flag_list = (int32_t*)p;
    A.nq = nq; A.nt = nt; A.idx2 = idx2; A.dist2 = dist2;
    if (hipMemsetAsync(A.flag_n, 0, sizeof(int32_t), st) != hipSuccess) return VO_EHIP;
    hipLaunchKernelGGL(k_bf_prep, dim3(((int64_t)B * qcap + 3) / 4), dim3(256), 0, st, q, nq, B, qcap, 2.f,
                       (__bf16*)A.qbf, (int32_t*)A.qn);
    hipLaunchKernelGGL(k_bf_prep, dim3(((int64_t)B * tcap + 3) / 4), dim3(256), 0, st, t, nt, B, tcap, 1.f,
                       (__bf16*)A.tbf, (int32_t*)A.tn);
    const int nqb = (qcap + BF_QB - 1) / BF_QB;
    hipLaunchKernelGGL(k_bf_mfma, dim3(B * nqb * A.tsplit), dim3(256), 0, st, A);
    hipLaunchKernelGGL(k_bf_merge, dim3(((int64_t)B * qcap + 255) / 256), dim3(256), 0, st, A);
    hipLaunchKernelGGL(k_bf_fixup, dim3(64), dim3(256), 0, st, A, q, t);
    return hipGetLastError() == hipSuccess ? VO_OK : VO_EHIP;
}
