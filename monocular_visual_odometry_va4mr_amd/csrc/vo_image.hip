// Image-side kernels for gfx950: pyramid ingest + pyrDown, Scharr derivatives,
// pyramidal Lucas-Kanade (one 64-lane wave per point), tracking compaction, and
// goodFeaturesToTrack (integer-exact min-eigenvalue map, 3x3 NMS, paged radix-select +
// LDS bitonic sort, wave-parallel greedy min-distance selection).
//
// Reference call sites: VisualOdometryPipeLine.py:256 (goodFeaturesToTrack),
// :281,:287 (calcOpticalFlowPyrLK).  Arithmetic follows oracle/vo_oracle_img.c
// operation by operation (that file restates OpenCV 4.6), so the
// integer stages are bit-exact and the float stages use the same op order (built with
// -ffp-contract=off, correctly rounded f32 div/sqrt).
#include "vo_dev.h"
#include <stdlib.h>

#include <float.h>
#include <math.h>
#include <type_traits>

namespace {

// ------------------------------------------------------------------ pyramid
// Levels are stored with a materialised VO_BORDER reflect-101 border and a 64-byte-multiple
// pitch.  One wave per row (256-thread blocks cover 4 rows); every lane writes an aligned
// vector (16, 4 or 16 bytes).  Bytes between the padded width and the pitch may be written
// with don't-care values.

// One pyramid level and its Scharr derivatives in one pass (buildOpticalFlowPyramid +
// calcSharrDeriv semantics).  A 256-thread block owns a PT_W x PT_H tile of
// the padded level: it materialises the level's values (with the reflect-101 border and a
// 1-pixel halo) in LDS, writes the tile to the pyramid with dword stores, and computes the
// int16 (dx, dy) Scharr of the tile's interior pixels from the same LDS tile.
//  * level 0: the values are frame bytes at reflect-101 coordinates;
//  * level l >= 1: cv::pyrDown of level l-1 ([1 4 6 4 1]^2 / 256).  The source rectangle
//    under the tile is staged with aligned dword loads, filtered horizontally once per
//    staged row into LDS, then vertically per output pixel (exact integers; the order of
//    the two passes does not change the result).
// The derivative image's zero border is never written: the derivative buffers are
// zero-initialised and only interior pixels are stored (zeros fill partial vectors).
#define PT_W 128
#define PT_H 16
#ifndef PYR0_TH
#define PYR0_TH 32                          // level-0 tile rows
#endif
#define PV_W (PT_W + 8)                     // tile cols px0-4 .. px0+PT_W+3
#define PV_H (PT_H + 2)                     // tile rows py0-1 .. py0+PT_H
#define PS_H (2 * PV_H + 3)                 // staged source rows (level >= 1)
#define PS_W ((2 * PV_W + 3 + 8 + 3) / 4 * 4)  // staged source cols incl. dword alignment slack

struct PyrLevelArgs {
    const uint8_t* src;     // level 0: frames [B][H][W]; else the pyramid (level l-1 inside)
    int64_t sstride;        // per chain: frame bytes or pyramid stride
    int sw, sh, spitch;     // source level l-1 (level >= 1)
    int64_t soff;
    uint8_t* pyr;           // destination pyramid (level l)
    int64_t pstride;
    int16_t* der;           // destination derivatives (level l): interleaved (dx, dy) int16 pairs
    int64_t dstride;
    int w, h, pitch;
    int64_t off;
    int level;
};

// L0: level 0 (frame bytes; its instantiation carries no source-staging LDS, so more blocks
// fit per CU).  FSRC (pyrDown levels): the source level is level 0 read straight from the frame
// at reflect-101 coordinates -- the values level 0's materialised border holds -- so level 1
// needs no level-0 tile of another block (k_pyr01 builds both in one launch).
template <bool L0, int TH, bool FSRC>
VO_DEV void pyr_tile(const PyrLevelArgs& A, int px0, int py0)
{
    constexpr int PH = TH + 2, SH = 2 * PH + 3, RPT = TH / 8;   // tile rows + halo, staged source rows, rows / thread
    __shared__ uint32_t PVw[PH * PV_W / 4];
    __shared__ int yk[PH], xc[PV_W];
    __shared__ int mm[4];
    uint8_t* PV = (uint8_t*)PVw;
    const int tid = threadIdx.x;
    const int b = blockIdx.z;
    const int pw = A.w + 2 * VO_BORDER, ph = A.h + 2 * VO_BORDER;
    // level coordinates of the tile's rows / cols (-1: outside the padded level)
    if (tid < 4) mm[tid] = (tid & 1) ? -1 : 0x7fffffff;
    __syncthreads();
    if (tid < PH) {
        const int py = py0 - 1 + tid;
        const int y = (py >= 0 && py < ph) ? refl101(py - VO_BORDER, A.h) : -1;
        yk[tid] = y;
        if (y >= 0) { atomicMin(&mm[0], y); atomicMax(&mm[1], y); }
    }
    if (tid < PV_W) {
        const int px = px0 - 4 + tid;
        const int x = (px >= 0 && px < pw) ? refl101(px - VO_BORDER, A.w) : -1;
        xc[tid] = x;
        if (x >= 0) { atomicMin(&mm[2], x); atomicMax(&mm[3], x); }
    }
    __syncthreads();
    // every load of a phase is issued before the first one is consumed (fixed trip counts,
    // unrolled): the staging is latency-bound otherwise
    constexpr int NPV = (PH * PV_W + 255) / 256;
    if constexpr (L0) {
        const uint8_t* fr = A.src + (int64_t)b * A.sstride;
        uint32_t v[NPV];
#pragma unroll
        for (int i = 0; i < NPV; ++i) {
            const int e = tid + 256 * i;
            // unconditional load from a clamped address (keeps the loads in one batch)
            const int ee = min(e, PH * PV_W - 1);
            const int k = ee / PV_W, c = ee - k * PV_W;
            const int y = yk[k], x = xc[c];
            v[i] = fr[(int64_t)max(y, 0) * A.w + max(x, 0)];
            if (y < 0 || x < 0) v[i] = 0;
        }
#pragma unroll
        for (int i = 0; i < NPV; ++i) {
            const int e = tid + 256 * i;
            if (e < PH * PV_W) PV[e] = (uint8_t)v[i];
        }
    } else {
        __shared__ uint32_t SRw[SH * PS_W / 4];
        __shared__ uint2 HSw[SH * PV_W / 4];                 // horizontal sums: u16 column quads
        const uint8_t* SR = (const uint8_t*)SRw;
        // source rectangle (level l-1 coordinates) under the tile
        const int sy0 = 2 * mm[0] - 2, sy1 = 2 * mm[1] + 2;
        const int sx0 = 2 * mm[2] - 2, sx1 = 2 * mm[3] + 2;
        const int nsr = sy1 - sy0 + 1;
        const int gx0 = sx0 + VO_BORDER;                 // padded source column of sx0
        const int ax0 = gx0 & ~3, sh = gx0 - ax0;
        const int nwd = (sx1 + VO_BORDER - ax0) / 4 + 1; // dwords per staged row
        constexpr int NSR = (SH * (PS_W / 4) + 255) / 256;
        uint32_t v[NSR];
        if constexpr (FSRC) {
            // staged byte j of row r = level-0 padded column ax0 + j = frame column
            // refl101(ax0 + j - VO_BORDER), frame row refl101(sy0 + r)
            const uint8_t* fr = A.src + (int64_t)b * A.sstride;
#pragma unroll
            for (int i = 0; i < NSR; ++i) {
                const int e = tid + 256 * i;
                const int r = e / (PS_W / 4), c = e - r * (PS_W / 4);
                const bool in = r < nsr && c < nwd;
                const uint8_t* row = fr + (int64_t)refl101(sy0 + (in ? r : 0), A.sh) * A.sw;
                const int cb = ax0 - VO_BORDER + 4 * (in ? c : 0);
                v[i] = (uint32_t)row[refl101(cb, A.sw)] | ((uint32_t)row[refl101(cb + 1, A.sw)] << 8) |
                       ((uint32_t)row[refl101(cb + 2, A.sw)] << 16) | ((uint32_t)row[refl101(cb + 3, A.sw)] << 24);
            }
        } else {
            const uint8_t* sbase = A.src + (int64_t)b * A.sstride + A.soff + ax0;
#pragma unroll
            for (int i = 0; i < NSR; ++i) {
                const int e = tid + 256 * i;
                const int r = e / (PS_W / 4), c = e - r * (PS_W / 4);
                const bool in = r < nsr && c < nwd;
                v[i] = *(const uint32_t*)(sbase + (int64_t)(sy0 + (in ? r : 0) + VO_BORDER) * A.spitch + 4 * (in ? c : 0));
            }
        }
#pragma unroll
        for (int i = 0; i < NSR; ++i) {
            const int e = tid + 256 * i;
            if (e < SH * (PS_W / 4)) SRw[e] = v[i];
        }
        __syncthreads();
        // horizontal [1 4 6 4 1] at the tile's columns, every staged row: four columns per
        // item.  Interior quads (four consecutive level columns) take their 11 source bytes
        // from four LDS dwords: byte-align to the first byte, then one v_dot4 per output with
        // weights (1,4,6,4) plus the fifth tap; quads that touch the reflect-101 border or
        // the outside of the level take the per-column path.
        static_assert(PV_W % 4 == 0, "pyrDown column quads");
        constexpr int PQ = PV_W / 4;
        uint2* HS2 = HSw;
        for (int e = tid; e < nsr * PQ; e += 256) {
            const int r = e / PQ, cq = e - r * PQ;
            const int x0 = xc[4 * cq], x3 = xc[4 * cq + 3];
            uint32_t o[4];
            if (x0 >= 0 && x3 == x0 + 3 && xc[4 * cq + 1] == x0 + 1 && xc[4 * cq + 2] == x0 + 2) {
                const int ob = r * PS_W + sh + (2 * x0 - 2 - sx0);
                const uint32_t* wp = SRw + (ob >> 2);
                const uint32_t sa = (uint32_t)(ob & 3);
                const uint32_t W0 = wp[0], W1 = wp[1], W2 = wp[2], W3 = wp[3];
                const uint32_t T0 = __builtin_amdgcn_alignbyte(W1, W0, sa);     // source bytes 0..3
                const uint32_t T1 = __builtin_amdgcn_alignbyte(W2, W1, sa);     // 4..7
                const uint32_t T2 = __builtin_amdgcn_alignbyte(W3, W2, sa);     // 8..11
                constexpr uint32_t K4 = 0x04060401u;                            // taps 1,4,6,4
                o[0] = __builtin_amdgcn_udot4(T0, K4, T1 & 0xffu, false);
                o[1] = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(T1, T0, 2), K4, (T1 >> 16) & 0xffu, false);
                o[2] = __builtin_amdgcn_udot4(T1, K4, T2 & 0xffu, false);
                o[3] = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(T2, T1, 2), K4, (T2 >> 16) & 0xffu, false);
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int x = xc[4 * cq + i];
                    o[i] = 0;
                    if (x >= 0) {
                        const uint8_t* q = SR + r * PS_W + sh + (2 * x - 2 - sx0);
                        o[i] = q[0] + 4 * q[1] + 6 * q[2] + 4 * q[3] + q[4];
                    }
                }
            }
            HS2[r * PQ + cq] = make_uint2(o[0] | (o[1] << 16), o[2] | (o[3] << 16));
        }
        __syncthreads();
        // vertical [1 4 6 4 1] + (acc + 128) >> 8 on packed column pairs: a horizontal sum is
        // <= 16 * 255 and a vertical one <= 65280, so the two 16-bit halves never carry into
        // each other (columns outside the level hold 0 and give 0)
        const uint2* HSq = HSw;
        for (int e = tid; e < PH * PQ; e += 256) {
            const int k = e / PQ, cq = e - k * PQ;
            const int y = yk[k];
            uint32_t v = 0;
            if (y >= 0) {
                const uint2* q = HSq + (2 * y - 2 - sy0) * PQ + cq;
                const uint2 q0 = q[0], q1 = q[PQ], q2 = q[2 * PQ], q3 = q[3 * PQ], q4 = q[4 * PQ];
                const uint32_t ax = q0.x + 4 * q1.x + 6 * q2.x + 4 * q3.x + q4.x + 0x00800080u;
                const uint32_t ay = q0.y + 4 * q1.y + 6 * q2.y + 4 * q3.y + q4.y + 0x00800080u;
                // bytes (ax >> 8), (ax >> 24), (ay >> 8), (ay >> 24)
                v = __builtin_amdgcn_perm(ay, ax, 0x07050301u);
            }
            PVw[k * (PV_W / 4) + cq] = v;
        }
    }    __syncthreads();
    // 4 pixels x RPT rows per thread: pyramid dword stores, then the Scharr of interior pixels
    const int tc = tid & 31, tr = tid >> 5;
    const int px = px0 + 4 * tc;
#pragma unroll
    for (int rr = 0; rr < RPT; ++rr) {
        const int k = 1 + RPT * tr + rr;
        const int py = py0 + RPT * tr + rr;
        if (py >= ph || px >= A.pitch) continue;
        const uint32_t* rowc = PVw + (k * PV_W) / 4 + 1 + tc;      // cols px..px+3
        *(uint32_t*)(A.pyr + (int64_t)b * A.pstride + A.off + (int64_t)py * A.pitch + px) = rowc[0];
        const int y = py - VO_BORDER, x0 = px - VO_BORDER;
        if (!A.der || y < 0 || y >= A.h || x0 + 3 < 0 || x0 >= A.w) continue;
        // rows k-1, k, k+1; bytes: col px-1 = byte 3 of dword [-1], px..px+3 = dword [0],
        // px+4 = byte 0 of dword [1]
        uint32_t o[4];
        const uint32_t* ru = rowc - PV_W / 4;
        const uint32_t* rl = rowc + PV_W / 4;
        const uint64_t U = ((uint64_t)ru[0] << 8) | (ru[-1] >> 24), L = ((uint64_t)rl[0] << 8) | (rl[-1] >> 24),
                       Cc = ((uint64_t)rowc[0] << 8) | (rowc[-1] >> 24);
        const uint64_t U5 = U | ((uint64_t)(ru[1] & 0xff) << 40), L5 = L | ((uint64_t)(rl[1] & 0xff) << 40),
                       C5 = Cc | ((uint64_t)(rowc[1] & 0xff) << 40);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            int dx = 0, dy = 0;
            const int x = x0 + i;
            if (x >= 0 && x < A.w) {
                const int ul = (int)((U5 >> (8 * i)) & 0xff), uc = (int)((U5 >> (8 * i + 8)) & 0xff),
                          ur = (int)((U5 >> (8 * i + 16)) & 0xff);
                const int ll = (int)((L5 >> (8 * i)) & 0xff), lc = (int)((L5 >> (8 * i + 8)) & 0xff),
                          lr = (int)((L5 >> (8 * i + 16)) & 0xff);
                const int cl = (int)((C5 >> (8 * i)) & 0xff), cr = (int)((C5 >> (8 * i + 16)) & 0xff);
                const int t0l = (ul + ll) * 3 + cl * 10;
                const int t0r = (ur + lr) * 3 + cr * 10;
                dx = t0r - t0l;
                dy = ((lr - ur) + (ll - ul)) * 3 + (lc - uc) * 10;
            }
            o[i] = (uint32_t)(uint16_t)(int16_t)dx | ((uint32_t)(uint16_t)(int16_t)dy << 16);
        }
        int16_t* dq = A.der + (int64_t)b * A.dstride + 2 * (A.off + (int64_t)py * A.pitch + px);
        *(uint4*)dq = make_uint4(o[0], o[1], o[2], o[3]);          // (dx, dy) of 4 pixels, 16 B
    }
}

template <bool L0, int TH>
__global__ void __launch_bounds__(256) k_pyr_level(PyrLevelArgs A)
{
    pyr_tile<L0, TH, false>(A, blockIdx.x * PT_W, blockIdx.y * TH);
}

// Levels 0 and 1 in one launch (few chains, where a launch is mostly latency): blocks with
// blockIdx.y < ty0 take level-0 tiles, the others level-1 tiles computed from the frame
// (pyr_tile FSRC); both grids' columns are covered by gridDim.x, surplus blocks exit.
__global__ void __launch_bounds__(256) k_pyr01(PyrLevelArgs A0, PyrLevelArgs A1, int tx0, int ty0, int tx1)
{
    if ((int)blockIdx.y < ty0) {
        if ((int)blockIdx.x < tx0) pyr_tile<true, PYR0_TH, false>(A0, blockIdx.x * PT_W, blockIdx.y * PYR0_TH);
    } else if ((int)blockIdx.x < tx1) {
        pyr_tile<false, PT_H, true>(A1, blockIdx.x * PT_W, (blockIdx.y - ty0) * PT_H);
    }
}

// k_pyr_rows<L0>: one pyramid level and its Scharr derivatives, streamed down the rows by
// single waves without LDS (round 5).  pyr_tile's blocks hold four wave slots and 25 KB of
// LDS each, so while another stream group's LK waves fill the CUs they wait for a CU to drain;
// a block of this kernel fits in the slot one finished LK wave frees.  A wave owns R level
// rows of a strip of 64 x 4 padded columns (lane = 4 consecutive columns; lanes 0 and 63 are
// halo lanes that only feed their neighbours' Scharr taps; strips step by PR_STEP columns and
// the last one is right-aligned, so it alone writes the right border):
//   level 0  row y is frame row y: two aligned dword loads and a byte align per lane (buffer
//            loads: a row end never reads past the frame buffer);
//   pyrDown  the horizontal [1 4 6 4 1] of source rows 2y-2 .. 2y+2 as packed u16 pairs (8
//            aligned source bytes per lane, the two outer taps from the neighbour lanes by DPP
//            wave shifts), kept in a five-row ring that advances two source rows per level
//            row, then the vertical taps and (acc + 128) >> 8 -- pyr_tile's integers exactly.
// Reflect-101 columns take their mirror column's byte by ds_bpermute inside the strip; the
// mirrored border rows are written by the wave that computes their source row; the Scharr of
// row y reads rows y-1, y, y+1 (the chunk's two halo rows evaluated on their own, reflect-101
// at the level's first and last row).  Same bytes and derivatives as pyr_tile.
#define PR_STEP 248
// one wave's item of a level: strip sx, rows sy R .. sy R + R - 1, chain b
template <bool L0>
VO_DEV void pyr_rows_wave(const PyrLevelArgs& A, int R, int sx, int sy, int b)
{
    const int lane = lane_id();
    const int wo = A.w, ho = A.h;
    const int pw = wo + 2 * VO_BORDER, ph = ho + 2 * VO_BORDER;
    const int pwa = (pw + 3) & ~3;
    const int ns = (pwa + PR_STEP - 1) / PR_STEP;
    const bool lastst = sx == ns - 1;
    const int base = lastst ? max(pwa - 252, -4) : sx * PR_STEP - 4;
    const int px = base + 4 * lane;
    const int y0 = sy * R;
    if (y0 >= ho || sx >= ns) return;
    const int y1 = min(y0 + R, ho);
    // columns this wave writes: [lo, hi); the earlier strips stop short of the last one's range,
    // so a border column and the Scharr taps next to it come from one wave only
    const int lo = lastst ? max(pwa - PR_STEP, 0) : sx * PR_STEP;
    const int hi = lastst ? pwa : min(sx * PR_STEP + PR_STEP, pwa - PR_STEP);
    const bool wlane = lane >= 1 && lane <= 62 && px >= lo && px < hi && px < pw;
    const bool dlane = wlane && px + 3 >= VO_BORDER && px < VO_BORDER + wo;
    // per byte of the lane: the strip position (lane * 4 + byte) holding its value
    int fsrc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c = px + j;
        const int sp = (c >= 0 && c < pw) ? VO_BORDER + refl101(c - VO_BORDER, wo) : c;
        const int rel = sp - base;
        fsrc[j] = (rel >= 0 && rel < 256) ? rel : 4 * lane + j;
    }
    const bool fixcols = base < VO_BORDER || base + 256 > VO_BORDER + wo;   // wave-uniform
    auto fix = [&](uint32_t v) -> uint32_t {
        if (!fixcols) return v;
        uint32_t o = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t t = (uint32_t)__builtin_amdgcn_ds_bpermute((fsrc[j] >> 2) << 2, (int)v);
            o |= ((t >> (8 * (fsrc[j] & 3))) & 0xffu) << (8 * j);
        }
        return o;
    };
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(A.src + (int64_t)b * A.sstride), (short)0, (int)A.sstride, 0x00020000);
    uint8_t* dst = A.pyr + (int64_t)b * A.pstride + A.off;
    // write level row y (+ the border rows that mirror it)
    auto put_row = [&](int y, uint32_t v) {
        if (!wlane) return;
        *(uint32_t*)(dst + (int64_t)(VO_BORDER + y) * A.pitch + px) = v;
        if (ho >= VO_BORDER + 2) {
            if (y >= 1 && y <= VO_BORDER) *(uint32_t*)(dst + (int64_t)(VO_BORDER - y) * A.pitch + px) = v;
            if (y >= ho - 1 - VO_BORDER && y <= ho - 2)
                *(uint32_t*)(dst + (int64_t)(VO_BORDER + 2 * ho - 2 - y) * A.pitch + px) = v;
        } else {
            for (int py = 0; py < ph; ++py) {
                if (py == VO_BORDER) py = VO_BORDER + ho;
                if (py < ph && refl101(py - VO_BORDER, ho) == y) *(uint32_t*)(dst + (int64_t)py * A.pitch + px) = v;
            }
        }
    };
    // Scharr of level row y from rows u = y-1, c = y, l = y+1 (calcSharrDeriv, as pyr_tile)
    auto put_der = [&](int y, uint32_t u, uint32_t c, uint32_t l) {
        const uint32_t ul = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x138, 0xF, 0xF, false);   // lane - 1
        const uint32_t cl = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0x138, 0xF, 0xF, false);
        const uint32_t ll = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)l, 0x138, 0xF, 0xF, false);
        const uint32_t ur = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x130, 0xF, 0xF, false);   // lane + 1
        const uint32_t cr = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0x130, 0xF, 0xF, false);
        const uint32_t lr = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)l, 0x130, 0xF, 0xF, false);
        if (!dlane || !A.der) return;
        const uint64_t U5 = ((uint64_t)u << 8) | (ul >> 24) | ((uint64_t)(ur & 0xff) << 40);
        const uint64_t L5 = ((uint64_t)l << 8) | (ll >> 24) | ((uint64_t)(lr & 0xff) << 40);
        const uint64_t C5 = ((uint64_t)c << 8) | (cl >> 24) | ((uint64_t)(cr & 0xff) << 40);
        uint32_t o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            int dx = 0, dy = 0;
            const int x = px + i - VO_BORDER;
            if (x >= 0 && x < wo) {
                const int uL = (int)((U5 >> (8 * i)) & 0xff), uc = (int)((U5 >> (8 * i + 8)) & 0xff),
                          uR = (int)((U5 >> (8 * i + 16)) & 0xff);
                const int lL = (int)((L5 >> (8 * i)) & 0xff), lc = (int)((L5 >> (8 * i + 8)) & 0xff),
                          lR = (int)((L5 >> (8 * i + 16)) & 0xff);
                const int cL = (int)((C5 >> (8 * i)) & 0xff), cR = (int)((C5 >> (8 * i + 16)) & 0xff);
                dx = ((uR + lR) * 3 + cR * 10) - ((uL + lL) * 3 + cL * 10);
                dy = ((lR - uR) + (lL - uL)) * 3 + (lc - uc) * 10;
            }
            o[i] = (uint32_t)(uint16_t)(int16_t)dx | ((uint32_t)(uint16_t)(int16_t)dy << 16);
        }
        int16_t* dq = A.der + (int64_t)b * A.dstride + 2 * (A.off + (int64_t)(VO_BORDER + y) * A.pitch + px);
        *(uint4*)dq = make_uint4(o[0], o[1], o[2], o[3]);
    };
    if constexpr (L0) {
        // frame row y: bytes px - B .. px - B + 3 (byte align shift uniform over the wave)
        auto ld_row = [&](int y, uint32_t& d0, uint32_t& d1) {
            const int ro = y * wo + base - VO_BORDER;
            const int al = (ro & ~3) + 4 * lane;
            d0 = __builtin_amdgcn_raw_buffer_load_b32(rs, al, 0, 0);
            d1 = __builtin_amdgcn_raw_buffer_load_b32(rs, al + 4, 0, 0);
        };
        auto val = [&](int y, uint32_t d0, uint32_t d1) {
            return fix(__builtin_amdgcn_alignbyte(d1, d0, (uint32_t)((y * wo + base - VO_BORDER) & 3)));
        };
        uint32_t a0, a1, c0, c1, n0, n1;
        const int yh = refl101(y0 - 1, ho);
        ld_row(yh, a0, a1);
        ld_row(y0, c0, c1);
        ld_row(y0 + 1 < y1 ? y0 + 1 : refl101(y1, ho), n0, n1);
        uint32_t vu = val(yh, a0, a1);
        uint32_t vc = val(y0, c0, c1);
        put_row(y0, vc);
        for (int y = y0; y < y1; ++y) {
            const int yn = y + 1 < y1 ? y + 1 : refl101(y1, ho);
            const uint32_t vl = val(yn, n0, n1);
            // the row after next, in flight while this row's Scharr runs
            const int y2 = y + 2 < y1 ? y + 2 : refl101(y1, ho);
            if (y + 1 < y1) ld_row(y2, n0, n1);
            if (y + 1 < y1) put_row(y + 1, vl);
            put_der(y, vu, vc, vl);
            vu = vc;
            vc = vl;
        }
    } else {
        const int loff = 2 * px - VO_BORDER;              // 8-aligned source column of byte 0
        auto ld_src = [&](int sr, uint32_t& d0, uint32_t& d1) {
            const int o = (int)A.soff + (VO_BORDER + sr) * A.spitch + loff;
            d0 = __builtin_amdgcn_raw_buffer_load_b32(rs, o, 0, 0);
            d1 = __builtin_amdgcn_raw_buffer_load_b32(rs, o + 4, 0, 0);
        };
        constexpr uint32_t K4 = 0x04060401u;               // taps 1, 4, 6, 4 (+ the fifth)
        auto hsum = [&](uint32_t D0, uint32_t D1, uint32_t& h01, uint32_t& h23) {
            const uint32_t L1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)D1, 0x138, 0xF, 0xF, false);   // lane - 1
            const uint32_t R0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)D0, 0x130, 0xF, 0xF, false);   // lane + 1
            const uint32_t o0 = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(D0, L1, 2), K4, (D0 >> 16) & 0xffu, false);
            const uint32_t o1 = __builtin_amdgcn_udot4(D0, K4, D1 & 0xffu, false);
            const uint32_t o2 = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(D1, D0, 2), K4, (D1 >> 16) & 0xffu, false);
            const uint32_t o3 = __builtin_amdgcn_udot4(D1, K4, R0 & 0xffu, false);
            h01 = o0 | (o1 << 16);
            h23 = o2 | (o3 << 16);
        };
        auto vert = [&](const uint32_t (&hx)[5], const uint32_t (&hy)[5]) {
            const uint32_t ax = hx[0] + 4 * hx[1] + 6 * hx[2] + 4 * hx[3] + hx[4] + 0x00800080u;
            const uint32_t ay = hy[0] + 4 * hy[1] + 6 * hy[2] + 4 * hy[3] + hy[4] + 0x00800080u;
            return fix(__builtin_amdgcn_perm(ay, ax, 0x07050301u));
        };
        // one level row on its own (the halo rows): five source rows, loads issued together
        auto direct = [&](int y) {
            uint32_t d[5][2], hx[5], hy[5];
#pragma unroll
            for (int k = 0; k < 5; ++k) ld_src(2 * y - 2 + k, d[k][0], d[k][1]);
#pragma unroll
            for (int k = 0; k < 5; ++k) hsum(d[k][0], d[k][1], hx[k], hy[k]);
            return vert(hx, hy);
        };
        uint32_t hx[5], hy[5];
        {
            uint32_t d[5][2];
#pragma unroll
            for (int k = 0; k < 5; ++k) ld_src(2 * y0 - 2 + k, d[k][0], d[k][1]);
#pragma unroll
            for (int k = 0; k < 5; ++k) hsum(d[k][0], d[k][1], hx[k], hy[k]);
        }
        uint32_t p0, p1, q0, q1;                           // source rows 2y+3, 2y+4, in flight
        ld_src(2 * y0 + 3, p0, p1);
        ld_src(2 * y0 + 4, q0, q1);
        uint32_t vu = direct(refl101(y0 - 1, ho));
        uint32_t vc = vert(hx, hy);
        put_row(y0, vc);
        for (int y = y0; y < y1; ++y) {
            uint32_t vl;
            if (y + 1 < y1) {
                hx[0] = hx[2]; hy[0] = hy[2];
                hx[1] = hx[3]; hy[1] = hy[3];
                hx[2] = hx[4]; hy[2] = hy[4];
                hsum(p0, p1, hx[3], hy[3]);
                hsum(q0, q1, hx[4], hy[4]);
                ld_src(2 * y + 5, p0, p1);
                ld_src(2 * y + 6, q0, q1);
                vl = vert(hx, hy);
                put_row(y + 1, vl);
            } else {
                vl = direct(refl101(y1, ho));
            }
            put_der(y, vu, vc, vl);
            vu = vc;
            vc = vl;
        }
    }
}

template <bool L0>
__global__ void __launch_bounds__(64) k_pyr_rows(PyrLevelArgs A, int R)
{
    pyr_rows_wave<L0>(A, R, (int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z);
}

// The small pyrDown levels of few chains in one launch (round 5): one 16-wave block per chain
// walks the levels in order, each wave taking (strip, row chunk) items of pyr_rows_wave, with a
// block barrier between levels (a level reads the one before).  At a few chains each level
// launch of k_pyr_rows was a ~12 us step of the frame's latency chain, mostly launch and
// dependency wait; the same items give the same bytes.
#define PYR_TAIL_MAX 6
struct PyrTailArgs {
    PyrLevelArgs a[PYR_TAIL_MAX];
    int R[PYR_TAIL_MAX];
    int n;
};
__global__ void __launch_bounds__(1024) k_pyr_tail(PyrTailArgs T)
{
    const int w = wave_id(), nw = (int)(blockDim.x >> 6);
    for (int l = 0; l < T.n; ++l) {
        const PyrLevelArgs& A = T.a[l];
        const int R = T.R[l];
        const int pwa = (A.w + 2 * VO_BORDER + 3) & ~3;
        const int ns = (pwa + PR_STEP - 1) / PR_STEP, nch = (A.h + R - 1) / R;
        for (int it = w; it < ns * nch; it += nw) pyr_rows_wave<false>(A, R, it % ns, it / ns, (int)blockIdx.x);
        __syncthreads();
    }
}

// Scharr (calcSharrDeriv) of one level: interleaved int16 (dx, dy) pairs, zero outside the
// image (the derivative image's constant border); 4 pixels (16 bytes) per lane
__global__ void __launch_bounds__(256) k_scharr(const uint8_t* __restrict__ pyr, int64_t pstride,
                                                int16_t* __restrict__ der, int64_t dstride,
                                                int w, int h, int pitch, int64_t off)
{
    const int b = blockIdx.z;
    const int px0 = (blockIdx.x * 64 + lane_id()) * 4;
    const int py = blockIdx.y * 4 + wave_id();
    if (px0 >= w + 2 * VO_BORDER || py >= h + 2 * VO_BORDER) return;
    const int y = py - VO_BORDER;
    const uint8_t* c = pyr + b * pstride + off + (int64_t)py * pitch;
    const uint8_t* u = c - pitch;   // reflect-101 border rows/cols are materialised
    const uint8_t* l = c + pitch;
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int px = px0 + k, x = px - VO_BORDER;
        int dx = 0, dy = 0;
        if (x >= 0 && x < w && y >= 0 && y < h) {
            const int t0l = (u[px - 1] + l[px - 1]) * 3 + c[px - 1] * 10;
            const int t0r = (u[px + 1] + l[px + 1]) * 3 + c[px + 1] * 10;
            const int t1l = l[px - 1] - u[px - 1], t1c = l[px] - u[px], t1r = l[px + 1] - u[px + 1];
            dx = t0r - t0l;
            dy = (t1r + t1l) * 3 + t1c * 10;
        }
        o[k] = (uint32_t)(uint16_t)(int16_t)dx | ((uint32_t)(uint16_t)(int16_t)dy << 16);
    }
    int16_t* dq = der + b * dstride + 2 * (off + (int64_t)py * pitch + px0);
    *(uint4*)dq = make_uint4(o[0], o[1], o[2], o[3]);
}

// ------------------------------------------------------------------ LK
struct LKParams {
    const uint8_t* prev;
    const int16_t* der;             // interleaved (dx, dy) int16 pairs, pixel o at der[2o], der[2o + 1]
    const uint8_t* next;
    int64_t pstride, dstride;
    int L;                          // top level used
    int lw[VO_MAX_LEVELS], lh[VO_MAX_LEVELS], lpitch[VO_MAX_LEVELS];
    int64_t loff[VO_MAX_LEVELS];
    int win_w, win_h, max_count;
    double eps2;
    float min_eig;
    // k_lk_w's convergence test decided in f32 where a margin settles it: fl32(ddx^2 + ddy^2)
    // <= eps2_lo means converged, >= eps2_hi not converged, anything between takes the exact
    // double test (fill_lk; both infinite when eps2 is too small for the f32 form)
    float eps2_lo, eps2_hi;
    // point segments: seg0 then seg1 (seg1 used only where its count > seg1_min)
    const float* p0;
    const int32_t* n0;
    int cap0;
    const float* p1;
    const int32_t* n1;
    int cap1;
    int seg1_min;
    const int32_t* chain_status;
    float* out;
    uint8_t* st;
    float* err;
    int ocap;
};

// Block -> (chain, point block).  With B >= 8 all blocks of one chain land on one XCD
// (hardware dispatch is round-robin over the 8 XCDs by linear block id), so the chain's
// pyramid level stays in that XCD's 4 MB L2 instead of being fetched by all eight.
// The mapping only affects speed; any block order gives the same results.
VO_DEV bool lk_block(int B, int nb, int& b, int& pb, bool xcd = true, int L = -1)
{
    if (L < 0) L = blockIdx.x;
    if (B >= 8 && xcd) {
        const int xcd = L & 7, k = L >> 3;
        b = xcd + 8 * (k / nb);
        pb = k % nb;
    } else {
        b = L / nb;
        pb = L % nb;
    }
    return b < B;
}

// One pyramid level of calcOpticalFlowPyrLK for every point (lkpyramid.cpp LKTrackerInvoker,
// SURVEY.md Appendix A): levels are separate launches, coarse to fine, and the point's
// running estimate lives in P.out between them (float, exactly as the in-register value).
// One wave per point; the 15x15 window is spread over the lanes (MAXJ pixels per lane).
// The next-image window moves every iteration, so each wave stages the J neighbourhood in
// LDS as packed 2x2 pixel quads (one ds_read_b32 = the four bilinear taps) and re-stages
// only when the estimate drifts more than M pixels.  The bilinear sum is two v_dot4_u32_u8
// over the 14-bit weights split into 7+7 bits; all window sums are integer and exact, so
// results match the CPU restatement bit for bit.
#define LK_M 4
// buffer resource over one chain's buffer: loads take 32-bit offsets (one VGPR, not a 64-bit
// address) and read zeros outside [0, bytes) instead of faulting
VO_DEV __amdgpu_buffer_rsrc_t lkq_rsrc(const void* base, int64_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}
#ifndef LK_JPRE
#define LK_JPRE 1
#endif
VO_DEV void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// a wave-uniform VALU result into an SGPR, where the arithmetic that consumes it (the weight
// packing) runs on the scalar unit instead of the VALU
VO_DEV int to_sgpr(int v)
{
    // an empty asm makes the VGPR value opaque, so the readfirstlane cannot be folded into the
    // conversion that produced it (an inline-asm readfirstlane instead broke LK on gfx950)
    asm volatile("" : "+v"(v));
    return __builtin_amdgcn_readfirstlane(v);
}
typedef short v2i16 __attribute__((ext_vector_type(2)));
VO_DEV v2i16 as_v2i16(uint32_t u) { return __builtin_bit_cast(v2i16, u); }
// v_dot2_i32_i16 (VOP3P) with its accumulator in an SGPR or as the inline constant 0: for a
// constant accumulator the compiler otherwise emits v_mov + v_dot2c (one VALU more)
VO_DEV int sdot2_sacc(uint32_t a, uint32_t b, int acc)
{
    int r;
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(acc));
    return r;
}
VO_DEV int sdot2_0(uint32_t a, uint32_t b)
{
    int r;
    asm("v_dot2_i32_i16 %0, %1, %2, 0" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
VO_DEV uint32_t v2u(v2i16 v) { return __builtin_bit_cast(uint32_t, v); }

// k_lk_w's bilinear weights w (0 .. 2^14) as an 8 + 7-bit split, bytes in the quad order of its J
// tile (w00, w10, w01, w11): wlo = w & 255, whi = w >> 8.  From the weights' low halves (the
// float bit patterns of w + 1.5 * 2^23 carry w in their low bits) two 16-bit packs and a few
// masks on the scalar unit (~10 SALU; the 7 + 7 form took ~25, and k_lk_w is SALU-bound).
VO_DEV void pack_w8_halves(uint32_t p0, uint32_t p1, uint32_t& wlo, uint32_t& whi)
{
    wlo = (p0 & 0x00ff00ffu) | ((p1 & 0x00ff00ffu) << 8);
    whi = ((p0 >> 8) & 0x00ff00ffu) | (p1 & 0xff00ff00u);
}
// operands in SGPRs (the iteration's weights): the two 16-bit packs as s_pack_ll_b32_b16
VO_DEV void pack_w8(uint32_t u00, uint32_t u01, uint32_t u10, uint32_t w11, uint32_t& wlo, uint32_t& whi)
{
    uint32_t p0, p1;                                         // (w00, w01), (w10, w11)
    asm("s_pack_ll_b32_b16 %0, %1, %2" : "=s"(p0) : "s"(u00), "s"(u01));
    asm("s_pack_ll_b32_b16 %0, %1, %2" : "=s"(p1) : "s"(u10), "s"(w11));
    pack_w8_halves(p0, p1, wlo, whi);
}
// any operands (the level-0 error pass)
VO_DEV void pack_w8_v(uint32_t w00, uint32_t w01, uint32_t w10, uint32_t w11, uint32_t& wlo, uint32_t& whi)
{
    pack_w8_halves((w00 & 0xffffu) | (w01 << 16), (w10 & 0xffffu) | (w11 << 16), wlo, whi);
}
VO_DEV uint32_t pack_w(int w00, int w01, int w10, int w11, int shift, int mask)
{
    return (uint32_t)((w00 >> shift) & mask) | ((uint32_t)((w01 >> shift) & mask) << 8) |
           ((uint32_t)((w10 >> shift) & mask) << 16) | ((uint32_t)((w11 >> shift) & mask) << 24);
}

template <int MAXJ>
__global__ void __launch_bounds__(64) k_lk(LKParams P, int level, int B, int nb)
{
    extern __shared__ uint32_t lk_tile[];
    int b, pb;
    if (!lk_block(B, nb, b, pb)) return;
    if (P.chain_status && P.chain_status[b] != 0) return;
    const int lane = lane_id();
    const int n0 = P.n0 ? P.n0[b] : 0;
    int n1 = P.n1 ? P.n1[b] : 0;
    if (n1 <= P.seg1_min) n1 = 0;
    const int ntot = n0 + n1;
    const int ww = P.win_w, wh = P.win_h, npx = ww * wh;
    const int TW = ww + 2 * LK_M, TH = wh + 2 * LK_M;
    uint32_t* tile = lk_tile + wave_id() * TW * TH;
    const float hx = (ww - 1) * 0.5f, hy = (wh - 1) * 0.5f;
    const int wpb = blockDim.x >> 6;
    const int cols = P.lw[level], rows = P.lh[level], pitch = P.lpitch[level];
    const int prow = rows + 2 * VO_BORDER;
    const uint8_t* I = P.prev + b * P.pstride + P.loff[level];
    const int16_t* DI = P.der + b * P.dstride + 2 * P.loff[level];
    const uint8_t* J = P.next + b * P.pstride + P.loff[level];
    const float sc = (float)(1. / (1 << level));
    // per-lane window slots: offsets in the level image and in the tile; slots past the
    // window read pixel (0,0) and are zeroed through their gradients / the error mask
    int goff[MAXJ], toff[MAXJ];
    bool live[MAXJ];
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
        const int k = lane + 64 * j;
        const int wy = k / ww, wx = k - wy * ww;
        live[j] = k < npx;
        goff[j] = live[j] ? wy * pitch + wx : 0;
        toff[j] = live[j] ? wy * TW + wx : 0;
    }
    for (int p = pb * wpb + wave_id(); p < ntot; p += nb * wpb) {
        const float* src = (p < n0) ? (P.p0 + ((int64_t)b * P.cap0 + p) * 2) : (P.p1 + ((int64_t)b * P.cap1 + (p - n0)) * 2);
        const int64_t oidx = (int64_t)b * P.ocap + p;
        const float ptx = src[0], pty = src[1];
        int status = 1;
        float errv = 0.f;
        float px = ptx * sc, py = pty * sc;
        float ox, oy;   // nextPts[ptidx]
        if (level == P.L) { ox = px; oy = py; }
        else { ox = P.out[2 * oidx] * 2.f; oy = P.out[2 * oidx + 1] * 2.f; }
        px -= hx;
        py -= hy;
        const int ipx = (int)floorf(px), ipy = (int)floorf(py);
        do {
            if (ipx < -ww || ipx >= cols || ipy < -wh || ipy >= rows) {
                if (level == 0) { status = 0; errv = 0.f; }
                break;
            }
            float a = px - ipx, bb = py - ipy;
            int iw00 = __float2int_rn((1.f - a) * (1.f - bb) * (float)(1 << 14));
            int iw01 = __float2int_rn(a * (1.f - bb) * (float)(1 << 14));
            int iw10 = __float2int_rn((1.f - a) * bb * (float)(1 << 14));
            int iw11 = (1 << 14) - iw00 - iw01 - iw10;
            int ival[MAXJ], ixv[MAXJ], iyv[MAXJ];
            int a11 = 0, a12 = 0, a22 = 0;
            const int64_t ib = (int64_t)(ipy + VO_BORDER) * pitch + (ipx + VO_BORDER);
#pragma unroll
            for (int j = 0; j < MAXJ; ++j) {
                const int64_t o = ib + goff[j];
                const uint8_t* s = I + o;
                const int16_t* d = DI + 2 * o;              // (dx, dy) pairs
                const int16_t* e = d + 1;
                const int v = DESCALE(__mul24(s[0], iw00) + __mul24(s[1], iw01) + __mul24(s[pitch], iw10) + __mul24(s[pitch + 1], iw11), 9);
                const int gx = DESCALE(__mul24(d[0], iw00) + __mul24(d[2], iw01) + __mul24(d[2 * pitch], iw10) + __mul24(d[2 * pitch + 2], iw11), 14);
                const int gy = DESCALE(__mul24(e[0], iw00) + __mul24(e[2], iw01) + __mul24(e[2 * pitch], iw10) + __mul24(e[2 * pitch + 2], iw11), 14);
                ival[j] = live[j] ? v : 0;
                ixv[j] = live[j] ? gx : 0;
                iyv[j] = live[j] ? gy : 0;
                a11 += __mul24(ixv[j], ixv[j]);
                a12 += __mul24(ixv[j], iyv[j]);
                a22 += __mul24(iyv[j], iyv[j]);
            }
            const int64_t iA11 = wave_sum_split(a11), iA12 = wave_sum_split(a12), iA22 = wave_sum_split(a22);
            const float FLT_SCALE = 1.f / (1 << 20);
            const float A11 = (float)iA11 * FLT_SCALE, A12 = (float)iA12 * FLT_SCALE, A22 = (float)iA22 * FLT_SCALE;
            float D = A11 * A22 - A12 * A12;
            const float minEig = (A22 + A11 - sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) / (float)(2 * ww * wh);
            if (minEig < P.min_eig || D < FLT_EPSILON) {
                if (level == 0) status = 0;
                break;
            }
            D = 1.f / D;
            float nx = ox - hx, ny = oy - hy;
            float pdx = 0.f, pdy = 0.f;
            int tx0 = -(1 << 30), ty0 = -(1 << 30);
            for (int it = 0; it < P.max_count; ++it) {
                const int inx = (int)floorf(nx), iny = (int)floorf(ny);
                if (inx < -ww || inx >= cols || iny < -wh || iny >= rows) {
                    if (level == 0) status = 0;
                    break;
                }
                if (inx < tx0 || inx > tx0 + 2 * LK_M || iny < ty0 || iny > ty0 + 2 * LK_M) {
                    // (re)stage the quad tile around the window; bytes outside the padded
                    // level are never read by an in-bounds window
                    tx0 = inx - LK_M;
                    ty0 = iny - LK_M;
                    __builtin_amdgcn_wave_barrier();
                    for (int q = lane; q < TW * TH; q += 64) {
                        const int r = q / TW, c = q - r * TW;
                        const int gy = ty0 + r + VO_BORDER, gx = tx0 + c + VO_BORDER;
                        uint32_t v = 0;
                        if (gy >= 0 && gy + 1 < prow && gx >= 0 && gx + 1 < pitch) {
                            const uint8_t* g = J + (int64_t)gy * pitch + gx;
                            v = (uint32_t)g[0] | ((uint32_t)g[1] << 8) | ((uint32_t)g[pitch] << 16) |
                                ((uint32_t)g[pitch + 1] << 24);
                        }
                        tile[q] = v;
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                }
                a = nx - inx;
                bb = ny - iny;
                iw00 = __float2int_rn((1.f - a) * (1.f - bb) * (float)(1 << 14));
                iw01 = __float2int_rn(a * (1.f - bb) * (float)(1 << 14));
                iw10 = __float2int_rn((1.f - a) * bb * (float)(1 << 14));
                iw11 = (1 << 14) - iw00 - iw01 - iw10;
                // iw00..iw10 are in [0, 2^14]; iw11 = 2^14 - (the others) can be -1, which
                // the unsigned dot cannot take: use iw11 + 1 and subtract the tap once
                const int neg = iw11 < 0;
                const int w11 = iw11 + neg;
                const uint32_t wlo = pack_w(iw00, iw01, iw10, w11, 0, 127);
                const uint32_t whi = pack_w(iw00, iw01, iw10, w11, 7, 255);
                const uint32_t* tb = tile + (iny - ty0) * TW + (inx - tx0);
                int b1 = 0, b2 = 0;
#pragma unroll
                for (int j = 0; j < MAXJ; ++j) {
                    const uint32_t q = tb[toff[j]];
                    uint32_t sum = (__builtin_amdgcn_udot4(q, whi, 0u, false) << 7) +
                                   __builtin_amdgcn_udot4(q, wlo, 256u, false);
                    if (neg) sum -= q >> 24;
                    const int diff = (int)(sum >> 9) - ival[j];
                    b1 += __mul24(diff, ixv[j]);      // |diff| <= 8160, |grad| <= 4080
                    b2 += __mul24(diff, iyv[j]);
                }
                // 32-bit reductions when every partial is below 2^24 (total < 2^30)
                const bool wide = __ballot((uint32_t)(b1 + (1 << 24)) >= (1u << 25) ||
                                           (uint32_t)(b2 + (1 << 24)) >= (1u << 25)) != 0;
                int64_t s1, s2;
                if (!wide) { s1 = wave_sum_dpp(b1); s2 = wave_sum_dpp(b2); }
                else { s1 = wave_sum_split(b1); s2 = wave_sum_split(b2); }
                const float fb1 = (float)s1 * FLT_SCALE;
                const float fb2 = (float)s2 * FLT_SCALE;
                const float ddx = (A12 * fb2 - A22 * fb1) * D;
                const float ddy = (A12 * fb1 - A11 * fb2) * D;
                nx += ddx;
                ny += ddy;
                ox = nx + hx;
                oy = ny + hy;
                if ((double)ddx * ddx + (double)ddy * ddy <= P.eps2) break;
                if (it > 0 && fabsf(ddx + pdx) < 0.01f && fabsf(ddy + pdy) < 0.01f) {
                    ox -= ddx * 0.5f;
                    oy -= ddy * 0.5f;
                    break;
                }
                pdx = ddx;
                pdy = ddy;
            }
            if (status && level == 0) {
                const float fx = ox - hx, fy = oy - hy;
                const int inx = (int)floorf(fx), iny = (int)floorf(fy);
                if (inx < -ww || inx >= cols || iny < -wh || iny >= rows) {
                    status = 0;
                    break;
                }
                const float aa = fx - inx, cc = fy - iny;
                iw00 = __float2int_rn((1.f - aa) * (1.f - cc) * (float)(1 << 14));
                iw01 = __float2int_rn(aa * (1.f - cc) * (float)(1 << 14));
                iw10 = __float2int_rn((1.f - aa) * cc * (float)(1 << 14));
                iw11 = (1 << 14) - iw00 - iw01 - iw10;
                const int64_t jb = (int64_t)(iny + VO_BORDER) * pitch + (inx + VO_BORDER);
                int es = 0;
#pragma unroll
                for (int j = 0; j < MAXJ; ++j) {
                    const uint8_t* s = J + jb + goff[j];
                    const int diff = DESCALE(__mul24(s[0], iw00) + __mul24(s[1], iw01) + __mul24(s[pitch], iw10) + __mul24(s[pitch + 1], iw11), 9) - ival[j];
                    es += live[j] ? (diff < 0 ? -diff : diff) : 0;
                }
                errv = (float)wave_sum_dpp(es) / (float)(32 * ww * wh);
            }
        } while (false);
        if (lane == 0) {
            P.out[2 * oidx] = ox;
            P.out[2 * oidx + 1] = oy;
            if (level == 0) {
                P.st[oidx] = (uint8_t)status;
                if (P.err) P.err[oidx] = errv;
            }
        }
    }
}

#ifdef VO_LK_PROF
// per level, per block (first 1024): start, end (wall clock, 100 MHz), iterations, J stagings,
// then wall-clock ticks spent in: I/dI staging, structure tensor, J staging, iterations
__device__ long long g_lkprof[VO_MAX_LEVELS][1024][8];
#define LKPROF_SET(k, v) do { if (lane == 0 && blockIdx.x < 1024) g_lkprof[level][blockIdx.x][k] = (v); } while (0)
#define LKPROF_ADD(k, v) do { if (lane == 0 && blockIdx.x < 1024) g_lkprof[level][blockIdx.x][k] += (v); } while (0)
#else
#define LKPROF_SET(k, v) do { } while (0)
#define LKPROF_ADD(k, v) do { } while (0)
#endif
#ifdef VO_LK_PROF
#define LKPROF_T(var) const long long var = wall_clock64()
#else
#define LKPROF_T(var) do { } while (0)
#endif

#ifdef VO_LK_CHECK
// diagnostics build: bounds-check every global load of k_lk_w against its chain's buffer;
// a bad address is reported and not dereferenced
#define LKCHK(ptr, base, bytes, what) \
    (((const char*)(ptr) >= (const char*)(base) && (const char*)(ptr) + 4 <= (const char*)(base) + (bytes)) ? true : \
     (printf("LKCHK %s b=%d p=%d level=%d off=%lld size=%lld\n", what, b, pcur, level, \
             (long long)((const char*)(ptr) - (const char*)(base)), (long long)(bytes)), false))
#else
#define LKCHK(ptr, base, bytes, what) true
#endif
#ifdef VO_LK_CHECK
// offset form for the buffer loads of k_lk_w (which read zeros past the chain's buffer)
#define LKCHKO(off, bytes, what) \
    do { if ((off) < 0 || (int64_t)(off) + 4 > (int64_t)(bytes)) \
        printf("LKCHK %s b=%d p=%d level=%d off=%lld size=%lld\n", what, b, pcur, level, (long long)(off), (long long)(bytes)); } while (0)
#else
#define LKCHKO(off, bytes, what) do { } while (0)
#endif

// ---------------------------------------------------------------------------------------
// k_lk_w<WW, WH>: the same LK level as k_lk for a compile-time window (the reference uses
// 15x15 for every dataset, main.py:36,66,96), with all window data staged through LDS by
// coalesced dword loads instead of per-lane byte gathers:
//   IR/DR  raw rows of I (u8) and dI (int16 pairs) under the (WW+1)x(WH+1) bilinear window,
//   QT     the J tile ((TW+1)x(TH+1), TW = WW + 2M) as packed 2x2 quads, read by the
//          iterations; built straight from registers (rows r and r + 1 loaded by every lane,
//          the next dword from the neighbouring lane): no raw-row LDS image.
// The tile origin is clamped so every staged row lies inside the padded level; dword rows
// may run up to 3 bytes past a row end (next row, or the >= 64-byte tail slack that the
// caller must leave after each pyramid -- launch_lk checks it).  Arithmetic is identical to
// k_lk (bit-exact with the CPU restatement).
template <int WW, int WH>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(8, 8))) k_lk_w(LKParams P, int level_hi, int level_lo, int B, int nb, int xcd)
{
    constexpr int WPB = 1;
    constexpr int NPX = WW * WH, MAXJ = (NPX + 63) / 64;
    constexpr int TW = WW + 2 * LK_M, TH = WH + 2 * LK_M;
    constexpr int JRW = (TW + 1 + 3 + 3) / 4, IRW = (WW + 1 + 3 + 3) / 4, DRW = WW + 1;
    constexpr int QM = (TW + 3) / 4, QS = 4 * QM;      // QT: quads of 4 columns, row stride QS
    // LDS rows: QT quads, the I window bytes and the dI dwords all have the row stride QS (in
    // their element), so one per-lane offset toff = row * QS + col indexes all three; J rows are
    // loaded as 8 dwords, so the staging lane -> (row, dword) map is (lane / 8, lane % 8)
    constexpr int IRS = QS / 4, JRS = 8;
    static_assert(JRW >= QM + 1 && JRW <= JRS && IRW <= IRS && IRW <= 8 && DRW == 16 && QS % 4 == 0,
                  "k_lk_w staging layout");
    // one spare row in QT / IR / DR: read (never used) by the dead lanes of window row 15
    __shared__ uint4 QT4_all[WPB][(TH + 1) * QM];
    __shared__ uint32_t IR_all[WPB][(WH + 2) * IRS];
    __shared__ uint32_t DR_all[WPB][(WH + 2) * QS];
    const int wv = WPB > 1 ? (int)(threadIdx.x >> 6) : 0;
    uint4* QT4 = QT4_all[wv];
    const uint32_t* QT = reinterpret_cast<const uint32_t*>(QT4);
    uint32_t* IR = IR_all[wv];
    uint32_t* DR = DR_all[wv];
    const uint8_t* ir8 = (const uint8_t*)IR;
    int b, pb, pcur = -1;
    const int lane = lane_id();
    int level = level_lo;
    LKPROF_SET(0, wall_clock64()); LKPROF_SET(1, 0);
    for (level = level_hi; level >= level_lo; --level)
        for (int k = 2; k < 8; ++k) LKPROF_SET(k, 0);
    level = level_lo;
    if (!lk_block(B, nb, b, pb, xcd != 0, (int)blockIdx.x * WPB + wv)) return;
    if (P.chain_status && P.chain_status[b] != 0) return;
    const int n0 = P.n0 ? P.n0[b] : 0;
    int n1 = P.n1 ? P.n1[b] : 0;
    if (n1 <= P.seg1_min) n1 = 0;
    const int ntot = n0 + n1;
    const float hx = (WW - 1) * 0.5f, hy = (WH - 1) * 0.5f;
    // held in registers: read from the kernel arguments inside the iteration loop it costs a
    // scalar load and its wait per iteration
    double eps2;
    asm volatile("" : "=s"(eps2) : "0"(P.eps2));
    float eps2_lo, eps2_hi;
    asm volatile("" : "=s"(eps2_lo) : "0"(P.eps2_lo));
    asm volatile("" : "=s"(eps2_hi) : "0"(P.eps2_hi));
    // window pixels of a lane: column lane % 16, rows 4 j + s with s = (lane / 32) + 2 (lane / 16
    // % 2), so that a 32-lane half reads rows s and s + 2 (row offsets 0 and 2 * QS = 48 dwords,
    // 16 banks apart: conflict-free) and pixel j sits at the constant offset toff + 4 j QS
    // (folded into the LDS instruction).  Column 15 and row 15 are dead lanes.
    static_assert(WW <= 16 && WH <= 16 && MAXJ == 4 && (2 * QS) % 32 == 16, "k_lk_w window map");
    const int wrow = ((lane >> 5) & 1) + 2 * ((lane >> 4) & 1), wcol = lane & 15;
    const int toff0 = wrow * QS + wcol;
    int toff[MAXJ];
    bool live[MAXJ];
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
        live[j] = wcol < WW && wrow + 4 * j < WH;
        toff[j] = toff0 + 4 * j * QS;
    }
    int tx0 = 0, ty0 = 0, jsh = 0;
    int cols = 0, rows = 0, pitch = 0, loff = 0;
    const __amdgpu_buffer_rsrc_t rI = lkq_rsrc(P.prev + (int64_t)b * P.pstride, P.pstride);
    const __amdgpu_buffer_rsrc_t rJ = lkq_rsrc(P.next + (int64_t)b * P.pstride, P.pstride);
    const __amdgpu_buffer_rsrc_t rD = lkq_rsrc(P.der + (int64_t)b * P.dstride, 2 * P.dstride);
    // Staging is split into issue (global loads into registers, fixed unrolled trip counts)
    // and store (LDS writes), so that every load of a stage is in flight at once: one memory
    // round trip per stage instead of one per loop trip.
    constexpr int NIR = ((WH + 1) * 8 + 63) / 64, NDR = ((WH + 1) * 16 + 63) / 64;
    constexpr int NJR = (TH * JRS + 63) / 64;             // 8 quad rows per load round
    // J tile origin covering the window at (inx, iny)
    auto j_origin = [&](int inx, int iny) {
        tx0 = max(inx - LK_M, -VO_BORDER);
        ty0 = min(max(iny - LK_M, -VO_BORDER), rows + VO_BORDER - 1 - TH);
        jsh = (tx0 + VO_BORDER) & 3;
    };
    // J rows r (a) and r + 1 (b) of the tile straight into registers, lane -> row 8 k + lane / 8
    // (+ 1 for b), aligned dword lane % 8 -- no raw-row LDS image: the quad build below takes
    // the dword to the right from the neighbouring lane (DPP) and row r + 1 from its own b load
    auto j_issue = [&](uint32_t (&v)[2][NJR]) {
        const int gx0 = tx0 + VO_BORDER, gy0 = ty0 + VO_BORDER;
        const int ln = lane;
        const int vo = loff + gy0 * pitch + (gx0 & ~3) + (ln >> 3) * pitch + 4 * (ln & 7);
#pragma unroll
        for (int k = 0; k < NJR; ++k) {
            v[0][k] = 0u;
            v[1][k] = 0u;
            if ((lane >> 3) + 8 * k < TH) {               // quad rows 0 .. TH - 1 use rows r, r + 1
                LKCHKO(vo + 8 * k * pitch + pitch, P.pstride, "J");
                v[0][k] = __builtin_amdgcn_raw_buffer_load_b32(rJ, vo, 8 * k * pitch, 0);
                v[1][k] = __builtin_amdgcn_raw_buffer_load_b32(rJ, vo, 8 * k * pitch + pitch, 0);
            }
        }
    };
    // the packed 2x2 quads QT: one item = quad row r, columns 4m..4m+3 (lane: r = 8 k + lane / 8,
    // m = lane % 8 < QM), built from the aligned dwords m, m + 1 of rows r and r + 1 (dword m + 1
    // from lane + 1 by DPP row_shl:1; m + 1 <= QM < 8 stays in the lane's 8-group) with byte-align
    // and two rounds of byte permutes, stored as one 16-B write; quad byte order (J[r][c],
    // J[r][c+1], J[r+1][c], J[r+1][c+1])
    auto j_store = [&](const uint32_t (&v)[2][NJR]) {
        const int ln = lane;
        const int m = ln & 7;
        const uint32_t jsel1 = (uint32_t)(jsh + 1) * 0x01010101u + 0x03020100u;   // bytes jsh+1 .. jsh+4
#pragma unroll
        for (int k = 0; k < NJR; ++k) {
            const uint32_t a0 = v[0][k], b0 = v[1][k];
            const uint32_t a1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a0, 0x101, 0xF, 0xF, false);   // row_shl:1
            const uint32_t b1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)b0, 0x101, 0xF, 0xF, false);
            const int r = (ln >> 3) + 8 * k;
#ifdef VO_LKX_NOQT
            if (false) {
#else
            if (m < QM && r < TH) {
#endif
                // row r bytes Wa0..Wa4 = bytes jsh .. jsh + 4 of (a1:a0), row r + 1 likewise Wb: A / C
                // hold W0..W3, Bv / D hold W1..W4 (byte-select by an SGPR selector, which also
                // covers jsh + 1 = 4); quad i = (Wa_i, Wb_i, Wa_i+1, Wb_i+1) (the weights' byte
                // order, pack_w8), one permute each
                const uint32_t A = __builtin_amdgcn_alignbyte(a1, a0, jsh);
                const uint32_t Bv = __builtin_amdgcn_perm(a1, a0, jsel1);
                const uint32_t C = __builtin_amdgcn_alignbyte(b1, b0, jsh);
                const uint32_t D = __builtin_amdgcn_perm(b1, b0, jsel1);
                QT4[r * QM + m] = make_uint4(__builtin_amdgcn_perm(C, A, 0x05010400u), __builtin_amdgcn_perm(C, A, 0x06020501u),
                                             __builtin_amdgcn_perm(C, A, 0x07030602u), __builtin_amdgcn_perm(D, Bv, 0x07030602u));
            }
        }
        wave_lds_sync();
    };
    // (re)stage the J tile so that it covers the window at (inx, iny)
    auto stage_j = [&](int inx, int iny) {
        LKPROF_ADD(3, 1);
        LKPROF_T(tj0);
        j_origin(inx, iny);
        uint32_t v[2][NJR];
        j_issue(v);
        wave_lds_sync();
        j_store(v);
        LKPROF_T(tj1);
        LKPROF_ADD(6, tj1 - tj0);
    };
    for (int p = pb + 0; p < ntot; p += nb) {
        const float* src = (p < n0) ? (P.p0 + ((int64_t)b * P.cap0 + p) * 2) : (P.p1 + ((int64_t)b * P.cap1 + (p - n0)) * 2);
        const int64_t oidx = (int64_t)b * P.ocap + p;
        pcur = p;
#ifdef VO_LK_CHECK
        if ((p < n0 && p >= P.cap0) || (p >= n0 && p - n0 >= P.cap1) || p >= P.ocap) {
            if (lane == 0) printf("LKCHK src b=%d p=%d n0=%d n1=%d\n", b, p, n0, n1);
            continue;
        }
#else
        (void)pcur;
#endif
        // per-point values are wave-uniform: keep them (and the addresses built from them)
        // in scalar registers
        const float ptx = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(src[0])));
        const float pty = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(src[1])));
        int status = 1;
        float errv = 0.f;
        float ox = 0.f, oy = 0.f;   // nextPts[ptidx]
        for (level = level_hi; level >= level_lo; --level) {
        cols = P.lw[level]; rows = P.lh[level]; pitch = P.lpitch[level]; loff = (int)P.loff[level];
        const unsigned colsW = (unsigned)(cols + WW), rowsW = (unsigned)(rows + WH);
        const float sc = __builtin_ldexpf(1.f, -level);     // 1 / 2^level, exact (no f64 division)
        float px = ptx * sc, py = pty * sc;
        if (level == P.L) { ox = px; oy = py; }
        else if (level == level_hi) {
            ox = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(P.out[2 * oidx]))) * 2.f;
            oy = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(P.out[2 * oidx + 1]))) * 2.f;
        } else {                // fused levels: the previous level's estimate, still in registers
            ox *= 2.f;
            oy *= 2.f;
        }
        px -= hx;
        py -= hy;
        const int ipx = (int)floorf(px), ipy = (int)floorf(py);
        do {
            if ((unsigned)(ipx + WW) >= colsW || (unsigned)(ipy + WH) >= rowsW) {   // outside the level
                if (level == 0) { status = 0; errv = 0.f; }
                break;
            }
            // stage I (u8) and dI (int16 x2) rows under the window, together with the J tile
            // of the first iteration (same bounds test as the iteration's): one round trip
            bool staged = false;
            {
                LKPROF_T(ti0);
                const int gx = ipx + VO_BORDER, gy = ipy + VO_BORDER;
                const int ish = gx & 3;
                const int ln = lane;
                const int vi = loff + gy * pitch + (gx & ~3) + (ln >> 3) * pitch + 4 * (ln & 7);   // 8 dwords / row
                // 16 (dx, dy) per row; lane -> row 4k + 2 ((ln >> 4) & 1) + (ln >> 5): the two rows a
                // 32-lane half stores are 2 apart (2 QS = 48 dwords, 16 banks), so the ds_write_b32
                // of DR below is conflict-free (rows r, r + 1 at QS = 24 collided 2-way)
                const int drow = 2 * ((ln >> 4) & 1) + (ln >> 5);
                const int vd = 4 * (loff + gy * pitch + gx + drow * pitch + (ln & 15));
                uint32_t vir[NIR], vdd[NDR], vjr[2][NJR];
#pragma unroll
                for (int k = 0; k < NIR; ++k) {
                    LKCHKO(vi + 8 * k * pitch, P.pstride, "I");
#ifdef VO_LKX_NOSTAGE
                    vir[k] = (uint32_t)(vi + k) * 0x01010101u;
#else
                    vir[k] = __builtin_amdgcn_raw_buffer_load_b32(rI, vi, 8 * k * pitch, 0);
#endif
                }
#pragma unroll
                for (int k = 0; k < NDR; ++k) {
                    LKCHKO(vd + 16 * k * pitch, 2 * P.dstride, "D");
#ifdef VO_LKX_NOSTAGE
                    vdd[k] = (uint32_t)(vd * 7 + k) & 0x00ff00ffu;
#else
                    vdd[k] = __builtin_amdgcn_raw_buffer_load_b32(rD, vd, 16 * k * pitch, 0);
#endif
                }
                {
                    const int jx = (int)floorf(ox - hx), jy = (int)floorf(oy - hy);
                    staged = LK_JPRE && (unsigned)(jx + WW) < colsW && (unsigned)(jy + WH) < rowsW && P.max_count > 0;
                    if (staged) {
                        LKPROF_ADD(3, 1);
                        j_origin(jx, jy);
                        j_issue(vjr);
                    } else {
                        tx0 = ty0 = -(1 << 28);        // no tile: the first iteration's test restages
                    }
                }
                wave_lds_sync();
#pragma unroll
                for (int k = 0; k < NIR; ++k) {
                    const int r = (ln >> 3) + 8 * k, c = ln & 7;
                    if (c < IRS) IR[r * IRS + c] = vir[k];
                }
#pragma unroll
                for (int k = 0; k < NDR; ++k) {
                    const int r = drow + 4 * k, c = ln & 15;
                    DR[r * QS + c] = vdd[k];
                }
                if (staged) j_store(vjr);      // syncs
                else wave_lds_sync();
                LKPROF_T(ti1);
                LKPROF_ADD(4, ti1 - ti0);
                float a = px - ipx, bb = py - ipy;
                const int iw00 = __float2int_rn((1.f - a) * (1.f - bb) * (float)(1 << 14));
                const int iw01 = __float2int_rn(a * (1.f - bb) * (float)(1 << 14));
                const int iw10 = __float2int_rn((1.f - a) * bb * (float)(1 << 14));
                const int iw11 = (1 << 14) - iw00 - iw01 - iw10;
                int ival[MAXJ], ixv[MAXJ], iyv[MAXJ];
                // dot accumulator seed 256 - 512 * I: the iteration's (bilinear sum + 256) >> 9 - I
                // becomes one arithmetic shift of the seeded sum (exact: the sum is >= 0 and
                // 512 * I is a multiple of the shift; the int32 result is in range)
                uint32_t iseed[MAXJ];
                int a11 = 0, a12 = 0, a22 = 0;
                // dI taps as int16 pairs against packed int16 weight pairs: two v_dot2_i32_i16
                // per sum (exact: |dI| <= 4080, weights <= 2^14)
                const v2i16 wp0 = as_v2i16((uint32_t)(iw00 & 0xffff) | ((uint32_t)iw01 << 16));
                const v2i16 wp1 = as_v2i16((uint32_t)(iw10 & 0xffff) | ((uint32_t)iw11 << 16));
#pragma unroll
                for (int j = 0; j < MAXJ; ++j) {
#ifdef VO_LKX_NOTENSOR
                    const uint32_t d00 = (uint32_t)(toff[j] * 977) & 0x03ff03ffu, d01 = d00 + 3, d10 = d00 + 5, d11 = d00 + 9;
                    const int v = (toff[j] * 31) & 8191;
#else
                    const uint8_t* s = ir8 + toff[j] + ish;
                    const uint32_t* d = DR + toff[j];
                    const uint32_t d00 = d[0], d01 = d[1], d10 = d[QS], d11 = d[QS + 1];
                    const int v = DESCALE(__mul24((int)s[0], iw00) + __mul24((int)s[1], iw01) +
                                          __mul24((int)s[QS], iw10) + __mul24((int)s[QS + 1], iw11), 9);
#endif
                    const int gx2 = __builtin_amdgcn_sdot2(as_v2i16(__builtin_amdgcn_perm(d11, d10, 0x05040100u)), wp1,
                                        sdot2_sacc(__builtin_amdgcn_perm(d01, d00, 0x05040100u), v2u(wp0), 1 << 13),
                                        false) >> 14;
                    const int gy2 = __builtin_amdgcn_sdot2(as_v2i16(__builtin_amdgcn_perm(d11, d10, 0x07060302u)), wp1,
                                        sdot2_sacc(__builtin_amdgcn_perm(d01, d00, 0x07060302u), v2u(wp0), 1 << 13),
                                        false) >> 14;
                    // a dead slot's I needs no mask: its gradients are zeroed below, so its
                    // mismatch never reaches b1 / b2 (|J - I| <= 8160 still fits the int16 pair),
                    // and the level-0 error masks it by live[j]
                    ival[j] = v;
                    iseed[j] = 256u - ((uint32_t)ival[j] << 9);
                    ixv[j] = live[j] ? gx2 : 0;
                    iyv[j] = live[j] ? gy2 : 0;
                }
                // the gradients as int16 pairs of pixels (0, 1) and (2, 3) (|dI| <= 4080): the
                // tensor here and the iteration's b1, b2 below are v_dot2_i32_i16 sums (exact)
                const v2i16 gxp0 = as_v2i16(__builtin_amdgcn_perm((uint32_t)ixv[1], (uint32_t)ixv[0], 0x05040100u));
                const v2i16 gxp1 = as_v2i16(__builtin_amdgcn_perm((uint32_t)ixv[3], (uint32_t)ixv[2], 0x05040100u));
                const v2i16 gyp0 = as_v2i16(__builtin_amdgcn_perm((uint32_t)iyv[1], (uint32_t)iyv[0], 0x05040100u));
                const v2i16 gyp1 = as_v2i16(__builtin_amdgcn_perm((uint32_t)iyv[3], (uint32_t)iyv[2], 0x05040100u));
                a11 = __builtin_amdgcn_sdot2(gxp0, gxp0, sdot2_0(v2u(gxp1), v2u(gxp1)), false);
                a12 = __builtin_amdgcn_sdot2(gxp0, gyp0, sdot2_sacc(v2u(gxp1), v2u(gyp1), 1 << 24), false);   // a12 + 2^24
                a22 = __builtin_amdgcn_sdot2(gyp0, gyp0, sdot2_0(v2u(gyp1), v2u(gyp1)), false);
                // one exact 32-bit reduction each when every lane has a11, a22 (>= 0) and the seeded
                // a12 below 2^25 (|a12| < 2^24): the 64 partials then sum below 2^31 (the a12 seeds
                // come off as 2^30); otherwise the split sums
                const bool twide = __ballot(max(max((uint32_t)a11, (uint32_t)a22), (uint32_t)a12) >= (1u << 25)) != 0;
                const float FLT_SCALE = 1.f / (1 << 20);
                float A11, A12, A22;
                if (!twide) {
                    wave_sum3_swap(a11, a22, a12);
                    A11 = (float)a11 * FLT_SCALE; A12 = (float)(a12 - (1 << 30)) * FLT_SCALE; A22 = (float)a22 * FLT_SCALE;
                } else {
                    A11 = (float)wave_sum_split(a11) * FLT_SCALE; A12 = (float)wave_sum_split(a12 - (1 << 24)) * FLT_SCALE;
                    A22 = (float)wave_sum_split(a22) * FLT_SCALE;
                }
                float D = A11 * A22 - A12 * A12;
                // minEig = (A22 + A11 - sqrtf(t)) / (2 WW WH) against min_eig: the correctly rounded
                // sqrt and division (~30 VALU) only where the raw v_sqrt_f32 (<= 2 ulp) and a
                // multiply by the reciprocal cannot settle the comparison.  Their error is below
                // 2^-21 (s + sum) / (2 WW WH) + 2^-21 |m|, inside the margin mg (exact decision).
                const float tq = (A11 - A22) * (A11 - A22) + 4.f * A12 * A12;
                const float sum2 = A22 + A11;
                const float sa = __builtin_amdgcn_sqrtf(tq);
                const float inv_n = 1.f / (float)(2 * WW * WH);
                const float ma = (sum2 - sa) * inv_n;
                const float mg = __builtin_fmaf(0x1p-20f, (sa + sum2) * inv_n + fabsf(ma), 0x1p-100f);
                bool reject;
                if (ma + mg < P.min_eig) reject = true;
                else if (ma - mg >= P.min_eig) reject = false;
                else reject = (sum2 - sqrtf(tq)) / (float)(2 * WW * WH) < P.min_eig;
                if (reject || D < FLT_EPSILON) {
                    if (level == 0) status = 0;
                    break;
                }
                D = 1.f / D;
                float nx = ox - hx, ny = oy - hy;
                float pdx = 0.f, pdy = 0.f;
                LKPROF_T(ta1);
                LKPROF_ADD(5, ta1 - ti1);
                for (int it = 0; it < P.max_count; ++it) {
                    // floor(n) as a float is exact, so n - floor(n) == n - (float)(int)floor(n)
                    const float fnx = floorf(nx), fny = floorf(ny);
                    const int inx = (int)fnx, iny = (int)fny;
                    // inx < -WW || inx >= cols || iny < -WH || iny >= rows, as two unsigned compares
                    if ((unsigned)(inx + WW) >= colsW || (unsigned)(iny + WH) >= rowsW) {
                        if (level == 0) status = 0;
                        break;
                    }
                    // (tx0, ty0 hold a far-away sentinel while no tile is staged at this level)
                    if ((unsigned)(inx - tx0) > 2u * LK_M || (unsigned)(iny - ty0) > 2u * LK_M) stage_j(inx, iny);
                    a = nx - fnx;
                    bb = ny - fny;
                    // wave-uniform weights: into scalar registers, packed by the scalar unit.
                    // cvRound(w) for w in [0, 2^14] is the low bits of the float w + 1.5 * 2^23
                    // (the add rounds half to even at unit spacing, as rint does), so one VALU add
                    // replaces round + convert; the bit fields the packing takes are those of w.
                    // (x * y) * 2^14 == (x * 2^14) * y exactly (power-of-two scaling, normal
                    // range), so the three products share two scaled factors.
                    const float LK_RND = 12582912.f;
                    const float xa = (1.f - a) * (float)(1 << 14), ya = 1.f - bb;
                    const uint32_t u00 = (uint32_t)to_sgpr(__float_as_int(xa * ya + LK_RND));
                    const uint32_t u01 = (uint32_t)to_sgpr(__float_as_int((a * (float)(1 << 14)) * ya + LK_RND));
                    const uint32_t u10 = (uint32_t)to_sgpr(__float_as_int(xa * bb + LK_RND));
                    const int w11 = (int)((1u << 14) + 3u * 0x4B400000u - u00 - u01 - u10);
                    // iw11 can be -1: dot with w11 + 1 and subtract the tap once
                    const int neg = w11 < 0;
                    uint32_t wlo, whi;
                    pack_w8(u00, u01, u10, (uint32_t)(w11 + neg), wlo, whi);
                    const uint32_t* tb = QT + (iny - ty0) * QS + (inx - tx0);
                    int b1 = 0, b2 = 0;
                    // all four quads read before the (wave-uniform) branch: one LDS round trip
                    uint32_t qv[MAXJ];
#pragma unroll
                    for (int j = 0; j < MAXJ; ++j) qv[j] = tb[toff[j]];
                    // the iw11 = -1 correction only in its own (wave-uniform) copy of the loop
                    auto mismatch = [&](auto negc) {
                        uint32_t dd[MAXJ];
#pragma unroll
                        for (int j = 0; j < MAXJ; ++j) {
                            const uint32_t q = qv[j];
                            uint32_t sum = (__builtin_amdgcn_udot4(q, whi, 0u, false) << 8) +
                                           __builtin_amdgcn_udot4(q, wlo, iseed[j], false);
                            if (decltype(negc)::value) sum -= q >> 24;
                            dd[j] = (uint32_t)((int)sum >> 9);       // |diff| <= 8160: an int16
                        }
                        // b1 = sum diff * Ix, b2 = sum diff * Iy as int16-pair dot products, each
                        // seeded with 2^24 (an SGPR operand): b' = b + 2^24
                        const uint32_t d01 = __builtin_amdgcn_perm(dd[1], dd[0], 0x05040100u);
                        const uint32_t d23 = __builtin_amdgcn_perm(dd[3], dd[2], 0x05040100u);
                        b1 = __builtin_amdgcn_sdot2(as_v2i16(d01), gxp0, sdot2_sacc(d23, v2u(gxp1), 1 << 24), false);
                        b2 = __builtin_amdgcn_sdot2(as_v2i16(d01), gyp0, sdot2_sacc(d23, v2u(gyp1), 1 << 24), false);
                    };
                    if (neg) mismatch(std::true_type());
                    else mismatch(std::false_type());
                    // |b| < 2^24 in every lane <=> b' in [0, 2^25): then the 64 seeded partials sum
                    // exactly in int32 (< 2^31) and the seeds come off as 64 * 2^24 = 2^30
                    const bool wide = __ballot(max((uint32_t)b1, (uint32_t)b2) >= (1u << 25)) != 0;
                    // int32 -> float and int64 -> float round the same integer identically
                    float fb1, fb2;
                    if (!wide) {
                        wave_sum2_swap(b1, b2);
                        fb1 = (float)(b1 - (1 << 30)) * FLT_SCALE; fb2 = (float)(b2 - (1 << 30)) * FLT_SCALE;
                    }
                    else {
                        fb1 = (float)wave_sum_split(b1 - (1 << 24)) * FLT_SCALE;
                        fb2 = (float)wave_sum_split(b2 - (1 << 24)) * FLT_SCALE;
                    }
                    const float ddx = (A12 * fb2 - A22 * fb1) * D;
                    const float ddy = (A12 * fb1 - A11 * fb2) * D;
                    nx += ddx;
                    ny += ddy;
                    ox = nx + hx;
                    oy = ny + hy;
                    // squares of floats are exact in double, so one fma rounds the same sum; the
                    // f32 form decides it outside the margin (P.eps2_lo / eps2_hi, fill_lk)
                    const float q2 = __builtin_fmaf(ddx, ddx, ddy * ddy);
                    if (q2 <= eps2_lo) break;
                    if (!(q2 >= eps2_hi)) {
                        const double dy2 = (double)ddy * ddy;
                        if (__builtin_fma((double)ddx, (double)ddx, dy2) <= eps2) break;
                    }
                    if (it > 0 && fabsf(ddx + pdx) < 0.01f && fabsf(ddy + pdy) < 0.01f) {
                        ox -= ddx * 0.5f;
                        oy -= ddy * 0.5f;
                        break;
                    }
                    pdx = ddx;
                    pdy = ddy;
                    LKPROF_ADD(2, 1);
                }
                {
                    LKPROF_T(te);
                    LKPROF_ADD(7, te - ta1);
                }
#ifdef VO_LKX_NOERR
                if (false) {
#else
                if (status && level == 0) {
#endif
                    const float fx = ox - hx, fy = oy - hy;
                    const int inx = (int)floorf(fx), iny = (int)floorf(fy);
                    if (inx < -WW || inx >= cols || iny < -WH || iny >= rows) {
                        status = 0;
                        break;
                    }
                    if ((unsigned)(inx - tx0) > 2u * LK_M || (unsigned)(iny - ty0) > 2u * LK_M) stage_j(inx, iny);
                    const float aa = fx - inx, cc = fy - iny;
                    const int w00 = __float2int_rn((1.f - aa) * (1.f - cc) * (float)(1 << 14));
                    const int w01 = __float2int_rn(aa * (1.f - cc) * (float)(1 << 14));
                    const int w10 = __float2int_rn((1.f - aa) * cc * (float)(1 << 14));
                    const int w11 = (1 << 14) - w00 - w01 - w10;
                    const int neg = w11 < 0;
                    uint32_t wlo, whi;
                    pack_w8_v((uint32_t)w00, (uint32_t)w01, (uint32_t)w10, (uint32_t)(w11 + neg), wlo, whi);
                    const uint32_t* tb = QT + (iny - ty0) * QS + (inx - tx0);
                    int es = 0;
#pragma unroll
                    for (int j = 0; j < MAXJ; ++j) {
                        const uint32_t q = tb[toff[j]];
                        uint32_t sum = (__builtin_amdgcn_udot4(q, whi, 0u, false) << 8) +
                                       __builtin_amdgcn_udot4(q, wlo, iseed[j], false);
                        if (neg) sum -= q >> 24;
                        const int diff = (int)sum >> 9;
                        es += live[j] ? (diff < 0 ? -diff : diff) : 0;
                    }
                    errv = (float)wave_sum_dpp(es) / (float)(32 * WW * WH);
                }
            }
        } while (false);
        }   // levels
        if (lane == 0) {
            P.out[2 * oidx] = ox;
            P.out[2 * oidx + 1] = oy;
            if (level_lo == 0) {
                P.st[oidx] = (uint8_t)status;
                if (P.err) P.err[oidx] = errv;
            }
        }
    }
    level = level_lo;
    LKPROF_SET(1, wall_clock64());
}

// ---------------------------------------------------- tracking compaction (:282-290)
// feature_tracking's status filtering (:283-290) as its own launch (vo_track); the engine's
// step runs the same block function at the start of the PnP block (vo_filter_pnp_triangulate)
__global__ void __launch_bounds__(256) k_track_compact(vo_dims d, vo_state s) { track_compact_block(d, s); }

// ------------------------------------------------------------------ GFTT
struct EigParams {
    const uint8_t* pyr;
    int64_t pstride;
    int W, H, pitch;
    int64_t off;
    int bs, harris;
    double harris_k;
    uint32_t* eig_max;
    uint64_t* keys;
    int32_t* nkeys;
    int ccap;
    int B, tiles_x, tiles_y;
    const int32_t* chain_status;
    float* eig_out;          // optional [B][W*H] eigen map (diagnostics, vo_gftt_eigmap)
};

// Fused cornerMinEigenVal / cornerHarris + 3x3 local-maximum test of goodFeaturesToTrack
// (featureselect.cpp, corner.cpp) on a 64x16 output tile.
//  * gradients: 3x3 Sobel (integer) at every covariance position, the covariance
//    position reflected (BORDER_REFLECT_101 of boxFilter) and Sobel reading the
//    materialised reflect-101 border of level 0;
//  * box sums of the gradient products (integer), lambda_min in double -> float;
//  * the eigen map is never stored: the tile recomputes a 1-pixel halo, and a pixel is a
//    candidate iff v > 0 and v >= its 8 neighbours.  With thr = quality * max >= 0 this is
//    exactly OpenCV's "v > thr and v == dilate(threshold(eig, thr))(x,y)"; the v > thr part
//    needs the global max and is applied by k_gftt_select.
//  * candidates are appended as (fkey(v) << 32 | y*W + x) with one atomic per block (the
//    list order is irrelevant: keys are unique and k_gftt_select orders them).
#define EIG_TW 64
#define EIG_TH 16
#define EIG_MAXBS 7
#define EIG_CW (EIG_TW + 2 + EIG_MAXBS - 1)
#define EIG_CH (EIG_TH + 2 + EIG_MAXBS - 1)
__global__ void __launch_bounds__(256) k_eignms(EigParams P)
{
    __shared__ int sdx[EIG_CW * EIG_CH];
    __shared__ int sdy[EIG_CW * EIG_CH];
    __shared__ float sE[(EIG_TH + 2) * (EIG_TW + 2)];
    __shared__ uint32_t smax;
    __shared__ int sh[16];
    __shared__ int sbase;
    const int ntile = P.tiles_x * P.tiles_y;
    const int item = xcd_item(blockIdx.x, P.B * ntile);
    if (item >= P.B * ntile) return;
    const int b = item / ntile, t = item - b * ntile;
    if (P.chain_status && P.chain_status[b] != 0) return;
    const int ty0 = t / P.tiles_x, tx0 = t - ty0 * P.tiles_x;
    const int x0 = tx0 * EIG_TW, y0 = ty0 * EIG_TH;
    const int bs = P.bs, a0 = bs / 2;
    const int ew = EIG_TW + 2, eh = EIG_TH + 2;          // eig region: tile + 1-px halo
    const int cw = ew + bs - 1, ch = eh + bs - 1;        // covariance region
    const uint8_t* img = P.pyr + b * P.pstride + P.off;
    if (threadIdx.x == 0) smax = 0;
    for (int q = threadIdx.x; q < cw * ch; q += blockDim.x) {
        const int qy = q / cw, qx = q - qy * cw;
        const int cx = refl101(x0 - 1 - a0 + qx, P.W), cy = refl101(y0 - 1 - a0 + qy, P.H);
        const uint8_t* c = img + (int64_t)(cy + VO_BORDER) * P.pitch + (cx + VO_BORDER);
        const uint8_t* u = c - P.pitch;
        const uint8_t* l = c + P.pitch;
        sdx[q] = (u[1] - u[-1]) + 2 * (c[1] - c[-1]) + (l[1] - l[-1]);
        sdy[q] = (l[-1] - u[-1]) + 2 * (l[0] - u[0]) + (l[1] - u[1]);
    }
    __syncthreads();
    const double s = 1.0 / ((double)(1 << 2) * bs * 255.0);
    uint32_t lmax = 0;
    for (int e = threadIdx.x; e < ew * eh; e += blockDim.x) {
        const int ey = e / ew, ex = e - ey * ew;
        int sxx = 0, sxy = 0, syy = 0;
        for (int i = 0; i < bs; ++i)
            for (int j = 0; j < bs; ++j) {
                const int q = (ey + i) * cw + (ex + j);
                const int gx = sdx[q], gy = sdy[q];
                sxx += gx * gx;
                sxy += gx * gy;
                syy += gy * gy;
            }
        float v;
        if (!P.harris) {
            const int64_t T = (int64_t)sxx + syy;
            const int64_t dd = (int64_t)sxx - syy;
            const int64_t Dd = dd * dd + 4 * (int64_t)sxy * sxy;
            v = (float)(((double)T - sqrt((double)Dd)) * (s * s * 0.5));
        } else {
            const int64_t det = (int64_t)sxx * syy - (int64_t)sxy * sxy;
            const int64_t T = (int64_t)sxx + syy;
            v = (float)(((double)det - P.harris_k * (double)(T * T)) * (s * s * s * s));
        }
        sE[e] = v;
        // the global max counts each image pixel once: the tile's own pixels only
        const int x = x0 - 1 + ex, y = y0 - 1 + ey;
        if (ex >= 1 && ex <= EIG_TW && ey >= 1 && ey <= EIG_TH && x < P.W && y < P.H) {
            const uint32_t k = fkey(v);
            lmax = k > lmax ? k : lmax;
            if (P.eig_out) P.eig_out[(int64_t)b * P.W * P.H + (int64_t)y * P.W + x] = v;
        }
    }
    // wave max, then one LDS atomic per wave
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const uint32_t t2 = __shfl_xor(lmax, o, 64);
        lmax = t2 > lmax ? t2 : lmax;
    }
    __syncthreads();
    if (lane_id() == 0 && lmax) atomicMax(&smax, lmax);
    if (!P.keys) {
        __syncthreads();
        if (threadIdx.x == 0 && smax) atomicMax(&P.eig_max[b], smax);
        return;
    }
    // local maxima among the tile's interior pixels (4 per thread)
    uint64_t kk[4];
    int cnt = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int k = threadIdx.x + 256 * j;
        const int ly = k / EIG_TW, lx = k - ly * EIG_TW;
        const int x = x0 + lx, y = y0 + ly;
        kk[j] = 0;
        if (x >= 1 && x < P.W - 1 && y >= 1 && y < P.H - 1) {
            const float* r = sE + ly * ew + lx;      // row above, centred at lx+1
            const float v = r[ew + 1];
            if (v > 0.f && v >= r[0] && v >= r[1] && v >= r[2] && v >= r[ew] && v >= r[ew + 2] &&
                v >= r[2 * ew] && v >= r[2 * ew + 1] && v >= r[2 * ew + 2]) {
                kk[j] = ((uint64_t)fkey(v) << 32) | (uint32_t)(y * P.W + x);
                ++cnt;
            }
        }
    }
    int tot;
    const int pre = block_scan_i32(cnt, sh, &tot);
    if (threadIdx.x == 0) {
        sbase = tot ? atomicAdd(&P.nkeys[b], tot) : 0;
        if (smax) atomicMax(&P.eig_max[b], smax);
    }
    __syncthreads();
    int pos = sbase + pre;
    uint64_t* out = P.keys + (int64_t)b * P.ccap;
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (kk[j]) {
            if (pos < P.ccap) out[pos] = kk[j];
            ++pos;
        }
}

// ---------------------------------------------------------------------------------------
// k_eig3: the fused min-eigenvalue + 3x3 local-maximum pass of k_eignms, specialised to the
// reference's configuration (blockSize 3, useHarrisDetector False; main.py:31-33,61-63,91-93)
// as a row-streaming kernel.  One wave owns an E3_OUT-column x E3_TH-row tile; lane = image
// column (3 halo lanes each side) and the wave slides down the rows keeping every
// intermediate in registers: the Sobel row terms of the last two image rows, the box row
// sums of the last two gradient rows, the last two eigen rows.  Horizontal neighbours come
// from the adjacent lanes through DPP wave shifts.  Integers, the double expression of
// lambda_min, the reflect-101 handling and the emitted key set are those of k_eignms (the
// parity tests compare corner lists and eigen maps bit for bit).  Keys are gathered in an
// LDS buffer and appended with one atomic per E3_CAP-sized batch.
#define E3_OUT 58
#define E3_TH 64
#define E3_CAP 512

VO_DEV int dpp_from_left(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xF, 0xF, false); }   // lane i <- i-1
VO_DEV int dpp_from_right(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x130, 0xF, 0xF, false); }  // lane i <- i+1

// sqrt of a double holding an integer in [0, 2^53): the compiler's correctly rounded sequence
// (v_rsq_f64 + Newton steps with a final fma correction) without its range reduction for inputs
// below 2^-767 and its class fix-ups, which such inputs never need; 0 (rsq = inf) selects 0.
// Bit-identical to sqrt() there, ~5 instructions shorter per pixel in k_eig3.
VO_DEV double sqrt_int_f64(double x)
{
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = 0.5 * y;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    double d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    return x == 0.0 ? 0.0 : g;
}

__global__ void __launch_bounds__(64) k_eig3(EigParams P)
{
    __shared__ uint64_t kbuf[E3_CAP];
    const int tiles = P.tiles_x * P.tiles_y;
    const int item = xcd_item(blockIdx.x, P.B * tiles);
    if (item >= P.B * tiles) return;
    const int b = item / tiles, t = item - b * tiles;
    if (P.chain_status && P.chain_status[b] != 0) return;
    const int ty = t / P.tiles_x, tx = t - ty * P.tiles_x;
    const int x0 = tx * E3_OUT, y0 = ty * E3_TH;
    const int W = P.W, H = P.H;
    const int lane = lane_id();
    const int c = x0 - 3 + lane;                         // image column of this lane
    const int cl = min(c, W + 2);                        // loads stay inside the padded row
    const uint8_t* colp = P.pyr + (int64_t)b * P.pstride + P.off + (int64_t)VO_BORDER * P.pitch + VO_BORDER + cl;
    const int g0 = max(y0 - 2, 0), g1 = min(y0 + E3_TH + 1, H - 1);   // gradient / box rows
    const int e0 = max(y0 - 1, 0);                                     // first eigen row
    const int o0 = max(y0, 1), o1 = min(y0 + E3_TH, H - 1);            // NMS rows [o0, o1)
    const int m1 = min(y0 + E3_TH, H);                                 // own rows [y0, m1)
    const bool own = lane >= 3 && lane < 3 + E3_OUT && c < W;
    const bool nms_col = own && c >= 1 && c < W - 1;
    const bool hedge = x0 == 0 || x0 + E3_OUT + 3 > W - 1;             // tile reaches column 0 or W-1
    const double s = 1.0 / ((double)(1 << 2) * 3 * 255.0);
    const double sc = s * s * 0.5;
    uint32_t kmax = 0;
    int nbuf = 0;
    uint64_t* out = P.keys ? P.keys + (int64_t)b * P.ccap : nullptr;
    auto flush = [&]() {
        int base = 0;
        if (lane == 0) base = atomicAdd(&P.nkeys[b], nbuf);
        base = __builtin_amdgcn_readfirstlane(base);
        wave_lds_sync();
        for (int i = lane; i < nbuf; i += 64)
            if (base + i < P.ccap) out[base + i] = kbuf[i];
        wave_lds_sync();
        nbuf = 0;
    };
    int hsA = 0, hdA = 0, hsB = 0, hdB = 0;              // Sobel row terms of image rows ir-2, ir-1
    int xA = 0, yA = 0, zA = 0, xB = 0, yB = 0, zB = 0;  // box row sums (xx, xy, yy) of rows pr-2, pr-1
    float eA = 0.f, eB = 0.f;                            // eigen rows r-2, r-1
    // the NMS maxima of those rows, each formed once when its row is new: 3-neighbour max of
    // row r-2, left / right max of row r-1 (fmaxf is exact and order-free on these values)
    float mA3 = 0.f, mB2 = 0.f;
    // eigen row r from the box row sums of rows r-1, r, r+1; then the NMS of row r-1
    auto eig_row = [&](int r, int ax, int ay, int az, int bx, int by, int bz, int cx, int cy, int cz) {
        const int sxx = ax + bx + cx, sxy = ay + by + cy, syy = az + bz + cz;
        const int T = sxx + syy, dd = sxx - syy;
        const double Dd = (double)dd * (double)dd + 4.0 * ((double)sxy * (double)sxy);
        const float v = (float)(((double)T - sqrt_int_f64(Dd)) * sc);
        if (own && r >= y0 && r < m1) {
            const uint32_t k = fkey(v);
            kmax = k > kmax ? k : kmax;
            if (P.eig_out) P.eig_out[(int64_t)b * W * H + (int64_t)r * W + c] = v;
        }
        const int rn = r - 1;
        const int iV = __float_as_int(v);
        const float mV2 = fmaxf(__int_as_float(dpp_from_left(iV)), __int_as_float(dpp_from_right(iV)));
        if (rn >= o0 && rn < o1) {
            const float mV = fmaxf(mV2, v);
            const bool cand = nms_col && out && eB > 0.f && eB >= fmaxf(fmaxf(mA3, mV), mB2);
            const uint64_t m = __ballot(cand);
            if (m) {
                if (cand) {
                    const int pre = __popcll(m & ((1ull << lane) - 1ull));
                    kbuf[nbuf + pre] = ((uint64_t)fkey(eB) << 32) | (uint32_t)(rn * W + c);
                }
                nbuf += __popcll(m);
                if (nbuf > E3_CAP - 64) flush();
            }
        }
        mA3 = fmaxf(mB2, eB);
        mB2 = mV2;
        eA = eB;
        eB = v;
    };
    // image rows are loaded E3_PF rows ahead of their use (a register ring), so the row loop
    // does not wait a full memory round trip per row
    constexpr int E3_PF = 8;
    int pf[E3_PF];
    const int ir_end = g1 + 1;
#pragma unroll
    for (int k = 0; k < E3_PF; ++k) pf[k] = (g0 - 1 + k <= ir_end) ? colp[(int64_t)(g0 - 1 + k) * P.pitch] : 0;
    // rows in groups of E3_PF, unrolled: ring slot u holds row ir0 + u, and the row registers
    // (A / B rings) are renamed instead of moved every row
    for (int ir0 = g0 - 1; ir0 <= ir_end; ir0 += E3_PF) {
#pragma unroll
    for (int u = 0; u < E3_PF; ++u) {
        const int ir = ir0 + u;
        if (ir > ir_end) break;
        const int iv = pf[u];
        pf[u] = (ir + E3_PF <= ir_end) ? colp[(int64_t)(ir + E3_PF) * P.pitch] : 0;
        const int il = dpp_from_left(iv), irt = dpp_from_right(iv);
        const int hs = il + 2 * iv + irt, hd = irt - il;
        if (ir >= g0 + 1) {
            const int pr = ir - 1;                       // gradient row
            const int gx = hdA + 2 * hdB + hd, gy = hs - hsA;
            // |gx|, |gy| <= 4 * 255: 24-bit multiplies (full rate; v_mul_lo_u32 is quarter rate)
            const int pxx = __mul24(gx, gx), pxy = __mul24(gx, gy), pyy = __mul24(gy, gy);
            int lxx = dpp_from_left(pxx), lxy = dpp_from_left(pxy), lyy = dpp_from_left(pyy);
            int rxx = dpp_from_right(pxx), rxy = dpp_from_right(pxy), ryy = dpp_from_right(pyy);
            if (hedge) {                                 // boxFilter BORDER_REFLECT_101 in x
                if (c == 0) { lxx = rxx; lxy = rxy; lyy = ryy; }
                if (c == W - 1) { rxx = lxx; rxy = lxy; ryy = lyy; }
            }
            const int hx = lxx + pxx + rxx, hy = lxy + pxy + rxy, hz = lyy + pyy + ryy;
            // eigen row pr-1 (BORDER_REFLECT_101 in y: row -1 is row 1)
            const int r = pr - 1;
            if (r >= e0) {
                if (r == 0) eig_row(r, hx, hy, hz, xB, yB, zB, hx, hy, hz);
                else eig_row(r, xA, yA, zA, xB, yB, zB, hx, hy, hz);
            }
            if (pr == H - 1 && pr >= e0 && pr >= 1)      // last image row: row H is row H-2
                eig_row(pr, xB, yB, zB, hx, hy, hz, xB, yB, zB);
            xA = xB; yA = yB; zA = zB;
            xB = hx; yB = hy; zB = hz;
        }
        hsA = hsB; hdA = hdB;
        hsB = hs; hdB = hd;
    }
    }
    if (out && nbuf) flush();
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const uint32_t t2 = __shfl_xor(kmax, o, 64);
        kmax = t2 > kmax ? t2 : kmax;
    }
    if (lane == 0 && kmax) atomicMax(&P.eig_max[b], kmax);
}

// ---------------------------------------------------------------- GFTT selection
#define SEL_THREADS 512
#define PAGE 4096
#define ACC_MAX 8192
#define GRID_LDS_CELLS 22528

struct SelParams {
    uint64_t* keys;
    int32_t* nkeys;          // in: local maxima appended; out: how many passed the quality gate
    const uint32_t* eig_max;
    double quality;
    int ccap, W, H;
    int max_corners;
    double min_dist;
    float* corners;
    int32_t* ncorners;
    int mcap;
    uint32_t* gscratch;      // per-chain L2 grid when the LDS grid is too small ([B][W*H] u32)
    int acc_lds;             // accepted-corner slots in LDS (min(mcap, ACC_MAX))
    int grid_lds;            // grid cells held in LDS (0: grid in L2)
    int64_t gstride;
    int grid_glb;            // the parallel walk may keep its grid + cell lists in gscratch
    const int32_t* chain_status;
};

// A grid cell holds up to two accepted-corner indices (u16 each, 0xFFFF = empty); the
// geometric bound (cell = round(minDistance) <= minDistance + 0.5) allows at most two.
VO_DEV uint32_t cell_get(bool lds, uint32_t* lg, uint32_t* gg, int c)
{
    // the L2 copy is only written by atomics: read it at agent scope (past the CU's L1)
    return lds ? lg[c] : __hip_atomic_load(&gg[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
VO_DEV int head_get(bool lds, int* lh, int* gh, int c)
{
    return lds ? lh[c] : __hip_atomic_load(&gh[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the parallel walk's L2 grid + cell-list heads sit after the conflict lists in gscratch
#define SEL_GG_OFF (PAGE * 8)
VO_DEV void cell_set(bool lds, uint32_t* lg, uint32_t* gg, int c, uint32_t v)
{
    if (lds) lg[c] = v;
    else atomicExch(&gg[c], v);
}

// hist[dgt] += 1 for every lane with `on` (12-bit digits), as one LDS atomic per distinct digit
// of the wave: peer lanes found with bit-sliced ballots
VO_DEV void wave_hist_add12(int* hist, bool on, int dgt)
{
    uint64_t peers = __ballot(on);
#pragma unroll
    for (int bit = 0; bit < 12; ++bit) {
        const bool b = (dgt >> bit) & 1;
        const uint64_t bm = __ballot(b);
        peers &= b ? bm : ~bm;
    }
    if (on && __ffsll((unsigned long long)peers) - 1 == lane_id()) atomicAdd(&hist[dgt], __popcll(peers));
}


#ifdef VO_SELECT_PROF
__device__ long long g_selprof[16];
}  // namespace
// diagnostics build only (libvo_hip_selprof.so, tools/sel_prof.py): block 0's phase timestamps
// of the last k_gftt_select launch (100 MHz wall clock)
extern "C" int vo_select_prof_read(long long* out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_selprof), sizeof(long long) * 16) == hipSuccess ? 0 : -2;
}
namespace {
#define SELPROF(i) do { if (threadIdx.x == 0 && blockIdx.x == 0) g_selprof[i] = wall_clock64(); } while (0)
#else
#define SELPROF(i) do { } while (0)
#endif

template <int NT>
__global__ void __launch_bounds__(NT) k_gftt_select(SelParams P)
{
    // dynamic LDS sized by the host (vo_gftt): page | candidate xy | accepted xy | grid + cell
    // heads (if they fit) | two conflict slots per candidate
    extern __shared__ uint64_t sel_dyn[];
    uint64_t* page = sel_dyn;
    uint32_t* cand_xy = (uint32_t*)(sel_dyn + PAGE);
    uint32_t* acc_xy = cand_xy + PAGE;
    uint32_t* lgrid = acc_xy + P.acc_lds;
    int* head = (int*)(lgrid + P.grid_lds);
    // each candidate's first two earlier conflicts, in LDS (most have at most two); the rest of
    // its list (up to CONF_K) is in the per-chain global scratch
    uint16_t* cf2 = (uint16_t*)(head + P.grid_lds);
    __shared__ uint32_t round_xy[64];
    __shared__ int sh_int[16];
    __shared__ int sh_scan[16];
    __shared__ uint64_t sh_u64[4];
    const int b = blockIdx.x;
    if (P.chain_status[b] != 0) return;
    const int tid = threadIdx.x;
    SELPROF(0);
    const int nk_all = P.nkeys[b];
    if (nk_all > P.ccap) {
        if (tid == 0) P.ncorners[b] = -1;          // capacity: k_add_finish raises it
        return;
    }
    // quality gate of goodFeaturesToTrack: v > quality * max(eig)  (featureselect.cpp);
    // ordered in-place compaction of the passing keys
    uint64_t* keys = P.keys + (int64_t)b * P.ccap;
    const float thr = (float)((double)fkey_inv(P.eig_max[b]) * P.quality);
    const uint64_t lo = ((uint64_t)fkey(thr) + 1ull) << 32;
    int nk = 0;
    // eight consecutive keys per thread per pass (one block scan per 8 * NT keys); every key of
    // a pass is read before the scan's barrier, and writes never pass a later pass's reads
    constexpr int KPT = 8;
    for (int base = 0; base < nk_all; base += NT * KPT) {
        const int i0 = base + tid * KPT;
        uint64_t kk[KPT];
        int cnt = 0;
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            kk[j] = i0 + j < nk_all ? keys[i0 + j] : 0ull;
            cnt += (i0 + j < nk_all && kk[j] >= lo) ? 1 : 0;
        }
        int tot;
        int pos = nk + block_scan_i32(cnt, sh_int, &tot);
#pragma unroll
        for (int j = 0; j < KPT; ++j)
            if (i0 + j < nk_all && kk[j] >= lo) keys[pos++] = kk[j];
        nk += tot;
    }
    __syncthreads();
    SELPROF(1);
    if (tid == 0) P.nkeys[b] = nk;
    const double md = P.min_dist;
    const bool use_grid = md >= 1;
    const int cs = use_grid ? __double2int_rn(md) : 1;
    const int gw = (P.W + cs - 1) / cs, gh = (P.H + cs - 1) / cs;
    const double md2 = md * md;
    const int want = P.max_corners > 0 ? P.max_corners : 0x7FFFFFFF;
    const int cap = P.mcap < P.acc_lds ? P.mcap : P.acc_lds;
    const int limit = want < cap ? want : cap;
    const bool lds = (int64_t)gw * gh <= P.grid_lds;
    // parallel walk: grid in LDS, or (P.grid_glb) grid + cell-list heads in gscratch
    const bool par = use_grid && (lds || P.grid_glb);
    uint32_t* gg = P.gscratch + (int64_t)b * P.gstride + (lds || !P.grid_glb ? 0 : SEL_GG_OFF);
    int* ghead = (int*)(gg + gw * gh);
    if (use_grid) {
        for (int q = tid; q < gw * gh; q += blockDim.x) cell_set(lds, lgrid, gg, q, 0xFFFFFFFFu);
        if (par && !lds)
            for (int q = tid; q < gw * gh; q += blockDim.x) atomicExch(&ghead[q], -1);
    }
    float* out = P.corners + (int64_t)b * P.mcap * 2;
    int nacc = 0;
    bool has_upper = false;
    uint64_t upper = 0;
    int remaining = nk;
    __syncthreads();
    while (remaining > 0 && nacc < limit) {
        // ---- this page: the min(PAGE, remaining) largest keys below `upper`
        uint64_t thr = 0;
        const int take = remaining < PAGE ? remaining : PAGE;
        if (remaining > PAGE) {
            // radix select of the PAGE-th largest key, 12-bit digits (histogram in the page
            // buffer, free until the gather): usually three passes over the keys instead of eight
            uint64_t prefix = 0, mask = 0;
            int k = PAGE;
            int* hist4 = (int*)page;
            for (int shift = 52; shift >= -8; shift -= 12) {
                const int sh = shift < 0 ? 0 : shift;                      // last digit: bits 3..0
                const int dbits = shift < 0 ? 4 : 12;
                const uint64_t dmask = ((uint64_t)1 << dbits) - 1;
                for (int q = tid; q < 4096; q += NT) hist4[q] = 0;
                __syncthreads();
                for (int i0 = tid; i0 < nk; i0 += 4 * NT) {
                    uint64_t kk[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) kk[u] = i0 + u * NT < nk ? keys[i0 + u * NT] : 0ull;
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const bool on = i0 + u * NT < nk && (!has_upper || kk[u] < upper) && (kk[u] & mask) == prefix;
                        wave_hist_add12(hist4, on, (int)((kk[u] >> sh) & dmask));
                    }
                }
                __syncthreads();
                // the digit holding the k-th largest: descending digit order over the threads,
                // NT / 4096-bin slices, one block scan
                constexpr int BPT = 4096 / NT;
                const int hi = 4095 - tid * BPT;
                int loc = 0;
#pragma unroll
                for (int j = 0; j < BPT; ++j) loc += hist4[hi - j];
                int tot;
                const int before = block_scan_i32(loc, sh_scan, &tot);
                if (before < k && k <= before + loc) {
                    int cum = before;
                    for (int j = 0; j < BPT; ++j) {
                        const int h = hist4[hi - j];
                        if (cum + h >= k) {
                            sh_u64[0] = prefix | ((uint64_t)(hi - j) << sh);
                            sh_int[0] = k - cum;
                            sh_int[1] = h;
                            break;
                        }
                        cum += h;
                    }
                }
                __syncthreads();
                prefix = sh_u64[0];
                k = sh_int[0];
                const int in_bucket = sh_int[1];
                mask |= dmask << sh;
                __syncthreads();
                if (in_bucket == k) break;          // the whole bucket is in: prefix (low bits 0) is the threshold
            }            thr = prefix;
        }
        if (tid == 0) sh_int[1] = 0;
        __syncthreads();
        for (int i0 = tid; i0 < nk; i0 += 4 * NT) {
            uint64_t kk[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) kk[u] = i0 + u * NT < nk ? keys[i0 + u * NT] : 0ull;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                // page order is irrelevant (sorted next): one LDS atomic per wave
                const bool on = i0 + u * NT < nk && (!has_upper || kk[u] < upper) && kk[u] >= thr;
                const uint64_t m = __ballot(on);
                if (m == 0) continue;
                const int leader = __ffsll((unsigned long long)m) - 1;
                int base = 0;
                if (lane_id() == leader) base = atomicAdd(&sh_int[1], __popcll(m));
                base = __shfl(base, leader, 64);
                const int pos = base + __popcll(m & ((1ull << lane_id()) - 1ull));
                if (on && pos < PAGE) page[pos] = kk[u];
            }
        }
        __syncthreads();
        for (int i = take + tid; i < PAGE; i += blockDim.x) page[i] = 0;
        __syncthreads();
        SELPROF(2);
        // ---- bitonic sort, descending (value desc, then larger address first)
        for (int size = 2; size <= PAGE; size <<= 1) {
            for (int stride = size >> 1; stride > 0; stride >>= 1) {
                for (int i = tid; i < PAGE / 2; i += blockDim.x) {
                    const int lo = 2 * i - (i & (stride - 1));
                    const int hi = lo + stride;
                    const bool desc = ((lo & size) == 0);
                    const uint64_t a = page[lo], c = page[hi];
                    if ((a < c) == desc) { page[lo] = c; page[hi] = a; }
                }
                __syncthreads();
            }
        }
        SELPROF(3);
        const uint64_t page_last = page[take - 1];
        if (par) {
            // ---- exact parallel form of OpenCV's sequential minDistance walk.  Candidate i
            // (rank order) is accepted iff no earlier accepted candidate in its 3x3 cell
            // neighbourhood is closer than minDistance, and no corner accepted on an earlier
            // page is.  Decisions only depend on earlier candidates, so they are resolved in
            // parallel rounds (each round decides at least the lowest undecided candidate);
            // the first `limit` accepted in rank order are the corners.
            for (int i = tid; i < take; i += blockDim.x) {
                const uint32_t addr = (uint32_t)page[i];
                const int y = (int)(addr / (uint32_t)P.W), x = (int)(addr - (uint32_t)y * P.W);
                cand_xy[i] = (uint32_t)x | ((uint32_t)y << 16);
            }
            // candidates by cell: with the grid in LDS, a counting sort (head[] = counts, then
            // start offsets; nxt[] = the candidate indices cell by cell), so a cell's candidates
            // are read with independent loads; otherwise linked lists in the L2 grid
            const int ncell = gw * gh;
            if (lds)
                for (int q = tid; q < ncell; q += blockDim.x) head[q] = 0;
            __syncthreads();
            int* nxt = (int*)page;                                // page keys are dead now
            volatile uint8_t* stt = (volatile uint8_t*)(nxt + PAGE);
            constexpr int CPT = PAGE / NT;                        // candidates per thread
            int slot[CPT];
#pragma unroll
            for (int kq = 0; kq < CPT; ++kq) {
                const int i = tid + kq * NT;
                if (i >= take) break;
                const uint32_t xy = cand_xy[i];
                const int x = (int)(xy & 0xFFFF), y = (int)(xy >> 16);
                const int xc = x / cs, yc = y / cs;
                bool rej = false;
                if (nacc > 0) {
                    const int x1 = max(xc - 1, 0), y1 = max(yc - 1, 0);
                    const int x2 = min(xc + 1, gw - 1), y2 = min(yc + 1, gh - 1);
                    for (int yy = y1; yy <= y2; ++yy)
                        for (int xx = x1; xx <= x2; ++xx) {
                            const uint32_t cv = cell_get(lds, lgrid, gg, yy * gw + xx);
                            for (int q = 0; q < 2; ++q) {
                                const uint32_t id = (cv >> (16 * q)) & 0xFFFFu;
                                if (id == 0xFFFFu) break;
                                const uint32_t aa = acc_xy[id];
                                const float ddx = (float)x - (float)(aa & 0xFFFF);
                                const float ddy = (float)y - (float)(aa >> 16);
                                if ((double)(ddx * ddx + ddy * ddy) < md2) rej = true;
                            }
                        }
                }
                stt[i] = rej ? 2 : 0;                             // 0 undecided, 1 accepted, 2 rejected
                if (lds) slot[kq] = atomicAdd(&head[yc * gw + xc], 1);
                else nxt[i] = atomicExch(&ghead[yc * gw + xc], i);
            }
            __syncthreads();
            if (lds) {
                // exclusive scan of the cell counts in place, then the cell-ordered index array
                const int cpt = (ncell + NT - 1) / NT, q0 = tid * cpt, q1 = min(q0 + cpt, ncell);
                int sum = 0;
                for (int q = q0; q < q1; ++q) sum += head[q];
                int tot;
                int run = block_scan_i32(sum, sh_int, &tot);
                for (int q = q0; q < q1; ++q) {
                    const int cnt = head[q];
                    head[q] = run;
                    run += cnt;
                }
                __syncthreads();
#pragma unroll
                for (int kq = 0; kq < CPT; ++kq) {
                    const int i = tid + kq * NT;
                    if (i >= take) break;
                    const uint32_t xy = cand_xy[i];
                    nxt[head[((int)(xy >> 16) / cs) * gw + (int)(xy & 0xFFFF) / cs] + slot[kq]] = i;
                }
                __syncthreads();
            }
            // visit(j) for every candidate j in cell cc, until it returns true
            auto for_cell = [&](int cc, auto&& visit) {
                if (lds) {
                    const int e0 = cc + 1 < ncell ? head[cc + 1] : take;
                    for (int k = head[cc]; k < e0; ++k)
                        if (visit(nxt[k])) return true;
                } else {
                    for (int j = head_get(false, head, ghead, cc); j >= 0; j = nxt[j])
                        if (visit(j)) return true;
                }
                return false;
            };
            // each candidate's earlier conflicts (same test as OpenCV's walk), found once:
            // count in LDS, indices in the per-chain scratch (the eigen-map buffer, unused on
            // this path); more than CONF_K conflicts -> rescan the cells in every round
            constexpr int CONF_K = 16;
            uint16_t* conf = (uint16_t*)(P.gscratch + (int64_t)b * P.gstride);
            uint8_t* ncf = (uint8_t*)(nxt + PAGE) + PAGE;          // PAGE bytes after stt
            for (int i = tid; i < take; i += blockDim.x) {
                if (stt[i] != 0) { ncf[i] = 0; continue; }
                const uint32_t xy = cand_xy[i];
                const int x = (int)(xy & 0xFFFF), y = (int)(xy >> 16);
                const int xc = x / cs, yc = y / cs;
                const int x1 = max(xc - 1, 0), y1 = max(yc - 1, 0);
                const int x2 = min(xc + 1, gw - 1), y2 = min(yc + 1, gh - 1);
                int c = 0;
                for (int yy = y1; yy <= y2; ++yy)
                    for (int xx = x1; xx <= x2; ++xx)
                        for_cell(yy * gw + xx, [&](int j) {
                            if (j >= i) return false;
                            const uint32_t aa = cand_xy[j];
                            const float ddx = (float)x - (float)(aa & 0xFFFF);
                            const float ddy = (float)y - (float)(aa >> 16);
                            if ((double)(ddx * ddx + ddy * ddy) < md2) {
                                if (c < 2) cf2[2 * i + c] = (uint16_t)j;
                                if (c < CONF_K) conf[(int64_t)i * CONF_K + c] = (uint16_t)j;
                                ++c;
                            }
                            return false;
                        });
                ncf[i] = (uint8_t)min(c, 255);
            }
            __syncthreads();
            SELPROF(5);
            for (;;) {
                if (tid == 0) sh_int[3] = 0;
                __syncthreads();
                bool changed = false;
                for (int i = tid; i < take; i += blockDim.x) {
                    if (stt[i] != 0) continue;
                    bool blocked = false, rej = false;
                    const int c = ncf[i];
                    if (c <= 2) {
                        for (int k = 0; k < c; ++k) {
                            const uint8_t sj = stt[cf2[2 * i + k]];
                            if (sj == 1) { rej = true; break; }
                            if (sj == 0) blocked = true;
                        }
                    } else if (c <= CONF_K) {
                        for (int k = 0; k < c; ++k) {
                            const uint8_t sj = stt[conf[(int64_t)i * CONF_K + k]];
                            if (sj == 1) { rej = true; break; }
                            if (sj == 0) blocked = true;
                        }
                    } else {
                        const uint32_t xy = cand_xy[i];
                        const int x = (int)(xy & 0xFFFF), y = (int)(xy >> 16);
                        const int xc = x / cs, yc = y / cs;
                        const int x1 = max(xc - 1, 0), y1 = max(yc - 1, 0);
                        const int x2 = min(xc + 1, gw - 1), y2 = min(yc + 1, gh - 1);
                        for (int yy = y1; yy <= y2 && !rej; ++yy)
                            for (int xx = x1; xx <= x2 && !rej; ++xx)
                                for_cell(yy * gw + xx, [&](int j) {
                                    if (j >= i) return false;
                                    const uint8_t sj = stt[j];
                                    if (sj == 2) return false;
                                    const uint32_t aa = cand_xy[j];
                                    const float ddx = (float)x - (float)(aa & 0xFFFF);
                                    const float ddy = (float)y - (float)(aa >> 16);
                                    if ((double)(ddx * ddx + ddy * ddy) < md2) {
                                        if (sj == 1) { rej = true; return true; }
                                        blocked = true;
                                    }
                                    return false;
                                });
                    }
                    if (rej) { stt[i] = 2; changed = true; }
                    else if (!blocked) { stt[i] = 1; changed = true; }
                }
                if (changed) sh_int[3] = 1;
                __syncthreads();
                const int any = sh_int[3];
                __syncthreads();
#ifdef VO_SELECT_PROF
                if (tid == 0 && blockIdx.x == 0) g_selprof[10]++;
#endif
                if (!any) break;
            }
            SELPROF(6);
            // accepted candidates in rank order -> corners (up to limit) and the grid
            for (int base = 0; base < take && nacc < limit; base += blockDim.x) {
                const int i = base + tid;
                const bool acc = i < take && stt[i] == 1;
                int tot;
                const int pos = nacc + block_scan_flag(acc, sh_int, &tot);
                if (acc && pos < limit) {
                    const uint32_t xy = cand_xy[i];
                    const int x = (int)(xy & 0xFFFF), y = (int)(xy >> 16);
                    acc_xy[pos] = xy;
                    out[2 * pos] = (float)x;
                    out[2 * pos + 1] = (float)y;
                    // at most two corners share a cell; slot order inside a cell is irrelevant
                    const int cell = (y / cs) * gw + (x / cs);
                    uint32_t cur = cell_get(lds, lgrid, gg, cell);
                    for (;;) {
                        const uint32_t nv = ((cur & 0xFFFFu) == 0xFFFFu) ? ((cur & 0xFFFF0000u) | (uint32_t)pos)
                                                                        : ((cur & 0xFFFFu) | ((uint32_t)pos << 16));
                        const uint32_t prev = lds ? atomicCAS(&lgrid[cell], cur, nv) : atomicCAS(&gg[cell], cur, nv);
                        if (prev == cur) break;
                        cur = prev;
                    }
                }
                nacc = min(nacc + tot, limit);
            }
            if (!lds) {
                // empty the cell lists this page used (the next page rebuilds them)
                for (int i = tid; i < take; i += blockDim.x) {
                    const uint32_t xy = cand_xy[i];
                    atomicExch(&ghead[((int)(xy >> 16) / cs) * gw + (int)(xy & 0xFFFF) / cs], -1);
                }
            }
            if (tid == 0) sh_int[2] = nacc;
        } else {
        // ---- greedy selection by wave 0, 64 candidates per round in sorted order.
            // A candidate survives if no accepted corner in the 3x3 neighbouring cells is closer
            // than minDistance (OpenCV's grid test).  Within a round, lane i additionally needs
            // every earlier accepted lane j < i of the round to pass the same test; the lanes
            // form a conflict mask against earlier tentative lanes, and wave-uniform scalar code
            // walks the tentative lanes in order to pick the accepted set -- exactly OpenCV's
            // sequential walk, without a ballot/shuffle round trip per accepted corner.
            if (wave_id() == 0) {
                const int lane = lane_id();
                for (int s0 = 0; s0 < take && nacc < limit; s0 += 64) {
                    const int i = s0 + lane;
                    bool tent = i < take;
                    int x = 0, y = 0;
                    if (tent) {
                        const uint32_t addr = (uint32_t)page[i];
                        y = (int)(addr / (uint32_t)P.W);
                        x = (int)(addr - (uint32_t)y * P.W);
                    }
                    const int xc = x / cs, yc = y / cs;
                    if (tent && use_grid) {
                        const int x1 = max(xc - 1, 0), y1 = max(yc - 1, 0);
                        const int x2 = min(xc + 1, gw - 1), y2 = min(yc + 1, gh - 1);
                        for (int yy = y1; yy <= y2 && tent; ++yy)
                            for (int xx = x1; xx <= x2 && tent; ++xx) {
                                const uint32_t cv = cell_get(lds, lgrid, gg, yy * gw + xx);
                                for (int q = 0; q < 2; ++q) {
                                    const uint32_t id = (cv >> (16 * q)) & 0xFFFFu;
                                    if (id == 0xFFFFu) break;
                                    const uint32_t a = acc_xy[id];
                                    const float ddx = (float)x - (float)(a & 0xFFFF);
                                    const float ddy = (float)y - (float)(a >> 16);
                                    if ((double)(ddx * ddx + ddy * ddy) < md2) { tent = false; break; }
                                }
                            }
                    }
                    const uint64_t tmask = __ballot(tent);
                    if (tmask == 0) continue;
                    uint64_t amask = tmask;
                    if (use_grid) {
                        // conflicts with earlier tentative lanes of this round
                        round_xy[lane] = (uint32_t)x | ((uint32_t)y << 16);
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                        uint32_t clo = 0, chi = 0;
                        uint64_t rest = tmask & ((1ull << lane) - 1ull) & (tent ? ~0ull : 0ull);
                        // uniform walk over the tentative lanes; each lane keeps the earlier ones
                        for (uint64_t m = tmask; m; m &= m - 1) {
                            const int j = __builtin_ctzll(m);
                            if (!((rest >> j) & 1ull)) continue;
                            const uint32_t a = round_xy[j];
                            const int tx = (int)(a & 0xFFFF), ty = (int)(a >> 16);
                            if (abs(tx / cs - xc) <= 1 && abs(ty / cs - yc) <= 1) {
                                const float ddx = (float)x - (float)tx, ddy = (float)y - (float)ty;
                                if ((double)(ddx * ddx + ddy * ddy) < md2) {
                                    if (j < 32) clo |= 1u << j; else chi |= 1u << (j - 32);
                                }
                            }
                        }
                        // in-order resolution on scalar registers
                        amask = 0;
                        for (uint64_t m = tmask; m; m &= m - 1) {
                            const int j = __builtin_ctzll(m);
                            const uint64_t cj = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)clo, j) |
                                                ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)chi, j) << 32);
                            if ((cj & amask) == 0) amask |= 1ull << j;
                        }
                    }
                    // respect maxCorners: keep the first (limit - nacc) accepted lanes
                    int nnew = __popcll(amask);
                    if (nnew > limit - nacc) {
                        uint64_t m = amask, keep = 0;
                        for (int c = 0; c < limit - nacc; ++c) { const uint64_t lb = m & (~m + 1ull); keep |= lb; m ^= lb; }
                        amask = keep;
                        nnew = limit - nacc;
                    }
                    if ((amask >> lane) & 1ull) {
                        const int idx = nacc + __popcll(amask & ((1ull << lane) - 1ull));
                        acc_xy[idx] = (uint32_t)x | ((uint32_t)y << 16);
                        out[2 * idx] = (float)x;
                        out[2 * idx + 1] = (float)y;
                        if (use_grid) {
                            // at most two corners share a cell; slot order inside a cell is irrelevant
                            const int cell = yc * gw + xc;
                            uint32_t cur = cell_get(lds, lgrid, gg, cell);
                            for (;;) {
                                const uint32_t nv = ((cur & 0xFFFFu) == 0xFFFFu) ? ((cur & 0xFFFF0000u) | (uint32_t)idx)
                                                                                : ((cur & 0xFFFFu) | ((uint32_t)idx << 16));
                                const uint32_t prev = lds ? atomicCAS(&lgrid[cell], cur, nv) : atomicCAS(&gg[cell], cur, nv);
                                if (prev == cur) break;
                                cur = prev;
                            }
                        }
                    }
                    nacc += nnew;
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                }
                if (lane == 0) sh_int[2] = nacc;
            }
        }
        __syncthreads();
        SELPROF(4);
        nacc = sh_int[2];
        upper = page_last;
        has_upper = true;
        remaining -= take;
        __syncthreads();
    }
    if (tid == 0) {
        // more corners wanted than this engine can hold -> never truncate silently.  The
        // status word is not written here: GFTT runs on a side stream concurrently with PnP,
        // which owns it; k_add_finish turns ncorners < 0 into VO_ST_CAPACITY.
        P.ncorners[b] = (nacc == cap && cap < want && remaining > 0) ? -1 : nacc;
    }
}

// ---------------------------------------------------------------- GFTT selection, split form
// (round 6).  k_gftt_select is one block per chain holding ~110 KB of LDS (C2) and 8-16 waves;
// beside the other stream group's LK flood -- one-wave blocks refilling every wave slot the
// moment it frees -- such a block starts only once a whole CU has drained (headline: 0.7 ms
// alone, 5-6 ms in the step).  The split form does the same selection in five LK-shaped
// launches: one-wave blocks, no LDS except the walk's 1.3 KB, so each block starts in the
// first wave slot that frees.
//   k_gsel_gate     many waves per chain: quality gate v > quality * max (featureselect.cpp),
//                   passing keys appended to the chain's list in any order, and a histogram of
//                   GS_NB value buckets (bucket = (key_max - fkey(v)) >> shift: descending
//                   value order, ~1/512 octave wide at C5);
//   k_gsel_scan     one wave per chain: exclusive scan of the histogram (bucket starts);
//   k_gsel_scatter  many waves per chain: every passing key to its bucket's range;
//   k_gsel_rank     many waves per chain: a key's final place = its bucket's start + the keys of
//                   its bucket larger than it (buckets hold ~1-70 keys: 12 at C2, 66 at C5), so
//                   the list ends fully sorted, descending u64 key = (value desc, then larger
//                   address first) as k_gftt_select's bitonic sort;
//   k_gsel_walk     one wave per chain: OpenCV's sequential minDistance walk over the sorted list,
//                   64 candidates per round (as the wave path of k_gftt_select): the accepted
//                   corners' cell grid holds each corner's offset inside its cell (no corner
//                   table), as u64 cells in the chain's eigen-map scratch; conflicts between the
//                   candidates of one round are found through a 128-entry LDS cell hash of lane
//                   masks (1.3 KB of LDS).
// The corner list is the one k_gftt_select produces (the GFTT parity tests run both forms).
// The split kernels do not read the chain status for their work (GFTT runs concurrently with
// PnP, which may change it mid-way, and the kernels must agree on what the histogram holds);
// only the walk skips writing corners for a chain that is no longer running, as k_gftt_select.
#define GS_NB 4096
#define GS_HASH 128

struct SelSplitParams {
    uint64_t* keys;          // gf_keys [B][ccap]: local maxima (in), then the bucket-grouped keys
    int32_t* nkeys;          // gf_n [B]: local maxima (in); passing keys (out, as k_gftt_select)
    const uint32_t* eig_max;
    double quality;
    int ccap, W, H;
    float invW;
    int want;                // maxCorners, 1 <= want <= mcap
    double md2;              // minDistance^2
    int cs, gw, gh;          // cell size cvRound(minDistance), grid
    uint32_t cs_m;           // ceil(2^32 / cs): x / cs = umulhi(x, cs_m) for x < 2^16
    float* corners;
    int32_t* ncorners;
    int mcap;
    uint64_t* sorted;        // gf_sort [B][sstride]: sorted keys [ccap] | histogram u32[GS_NB] | npass
    int64_t sstride;
    float* ggrid;            // u64 cell grid in the eigen-map scratch, 8-byte aligned
    int64_t gstride;         // floats per chain (W * H)
    int wpc;                 // waves per chain of gate / scatter / rank
    const int32_t* chain_status;
};

VO_DEV uint32_t* gs_hist(const SelSplitParams& P, int b) { return (uint32_t*)(P.sorted + (int64_t)b * P.sstride + P.ccap); }
VO_DEV int32_t* gs_npass(const SelSplitParams& P, int b) { return (int32_t*)(gs_hist(P, b) + GS_NB); }

// the chain's gate and bucket map: keys >= lo pass; bucket(k) = (kmax - (k >> 32)) >> shift
VO_DEV bool gs_range(const SelSplitParams& P, int b, uint64_t& lo, uint32_t& kmax, int& shift)
{
    kmax = P.eig_max[b];
    const float thr = (float)((double)fkey_inv(kmax) * P.quality);
    lo = ((uint64_t)fkey(thr) + 1ull) << 32;
    shift = 0;
    if ((uint64_t)kmax < (lo >> 32)) return false;
    const uint32_t R = kmax - (uint32_t)(lo >> 32);
    const int bits = R ? 32 - __clz(R) : 0;
    shift = bits > 12 ? bits - 12 : 0;
    return true;
}
VO_DEV int gs_bucket(uint64_t k, uint32_t kmax, int shift)
{
    const int q = (int)((kmax - (uint32_t)(k >> 32)) >> shift);
    return q < GS_NB - 1 ? q : GS_NB - 1;
}

__global__ void __launch_bounds__(64) k_gsel_gate(SelSplitParams P)
{
    const int b = blockIdx.x / P.wpc, w = blockIdx.x - b * P.wpc;
    const int nk_all = P.nkeys[b];
    if (nk_all > P.ccap) return;                         // capacity: the walk reports it
    uint64_t lo;
    uint32_t kmax;
    int sh;
    if (!gs_range(P, b, lo, kmax, sh)) return;
    const uint64_t* keys = P.keys + (int64_t)b * P.ccap;
    uint64_t* pass = P.sorted + (int64_t)b * P.sstride;
    uint32_t* hist = gs_hist(P, b);
    int32_t* npass = gs_npass(P, b);
    const int lane = lane_id();
    for (int base = w * 256; base < nk_all; base += P.wpc * 256) {
        uint64_t kk[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = base + u * 64 + lane;
            kk[u] = i < nk_all ? keys[i] : 0ull;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const bool on = kk[u] >= lo;                 // 0 (absent) never passes: lo >= 2^32
            const uint64_t m = __ballot(on);
            if (m == 0) continue;
            if (on) __hip_atomic_fetch_add(&hist[gs_bucket(kk[u], kmax, sh)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int leader = __ffsll((unsigned long long)m) - 1;
            int pos = 0;
            if (lane == leader) pos = atomicAdd(npass, __popcll(m));
            pos = __shfl(pos, leader, 64) + __popcll(m & ((1ull << lane) - 1ull));
            if (on) pass[pos] = kk[u];
        }
    }
}

__global__ void __launch_bounds__(64) k_gsel_scan(SelSplitParams P)
{
    const int b = blockIdx.x;
    uint32_t* hist = gs_hist(P, b);
    const int lane = lane_id();
    uint4* h4 = (uint4*)hist + lane * (GS_NB / 256);     // 64 consecutive bins per lane
    // two passes over the lane's bins (read to sum, re-read to write) keep it at <= 64 VGPRs, so
    // the wave fits the slot of one finished LK wave
    uint32_t sum = 0;
#pragma unroll
    for (int j = 0; j < GS_NB / 256; ++j) {
        const uint4 v = h4[j];
        sum += v.x + v.y + v.z + v.w;
    }
    // inclusive wave scan of the lane sums
    uint32_t inc = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
    }
    if (__ballot(sum != 0) == 0) return;                 // nothing passed (or the chain was skipped)
    uint32_t run = inc - sum;
#pragma unroll
    for (int j = 0; j < GS_NB / 256; ++j) {
        const uint4 v = h4[j];
        uint4 o;
        o.x = run; run += v.x;
        o.y = run; run += v.y;
        o.z = run; run += v.z;
        o.w = run; run += v.w;
        h4[j] = o;
    }
}

__global__ void __launch_bounds__(64) k_gsel_scatter(SelSplitParams P)
{
    const int b = blockIdx.x / P.wpc, w = blockIdx.x - b * P.wpc;
    const int n = *gs_npass(P, b);
    if (n == 0) return;
    uint64_t lo;
    uint32_t kmax;
    int sh;
    gs_range(P, b, lo, kmax, sh);
    const uint64_t* pass = P.sorted + (int64_t)b * P.sstride;
    uint32_t* hist = gs_hist(P, b);
    uint64_t* grouped = P.keys + (int64_t)b * P.ccap;
    for (int i = w * 64 + lane_id(); i < n; i += P.wpc * 64) {
        const uint64_t k = pass[i];
        const uint32_t pos = atomicAdd(&hist[gs_bucket(k, kmax, sh)], 1u);
        grouped[pos] = k;
    }
}

__global__ void __launch_bounds__(64) k_gsel_rank(SelSplitParams P)
{
    const int b = blockIdx.x / P.wpc, w = blockIdx.x - b * P.wpc;
    const int n = *gs_npass(P, b);
    if (n == 0) return;
    uint64_t lo;
    uint32_t kmax;
    int sh;
    gs_range(P, b, lo, kmax, sh);
    const uint32_t* hist = gs_hist(P, b);              // after the scatter: bucket ends
    const uint64_t* grouped = P.keys + (int64_t)b * P.ccap;
    uint64_t* sorted = P.sorted + (int64_t)b * P.sstride;
    for (int i = w * 64 + lane_id(); i < n; i += P.wpc * 64) {
        const uint64_t k = grouped[i];
        const int q = gs_bucket(k, kmax, sh);
        const int st = q ? (int)hist[q - 1] : 0, en = (int)hist[q];
        int cnt = 0;
        for (int j = st; j < en; ++j) cnt += grouped[j] > k ? 1 : 0;
        sorted[st + cnt] = k;
    }
}

// grid cells (u64 in the chain's eigen-map scratch): up to four corners, each stored as 1 + its
// offset inside the cell (ox | oy << 8).  Every access to the grid comes from this one wave, so
// all of them are atomics at workgroup scope (coherent among themselves by the memory model,
// served by the CU's own XCD instead of the device coherence point).  The grid stays out of
// LDS on purpose: beside the LK flood a block waits for a CU with that much LDS free (a 12 KB
// u16 cell table in LDS made the headline's walk 6-10 ms instead of 0.5 ms).
__global__ void __launch_bounds__(64) k_gsel_walk(SelSplitParams P)
{
    __shared__ uint64_t rhash[GS_HASH];
    __shared__ uint32_t rxy[64];
    const int b = blockIdx.x;
    const int lane = lane_id();
    // the histogram and the pass counter are this call's; zero them for the next one
    uint32_t* hist = gs_hist(P, b);
    int32_t* npass = gs_npass(P, b);
    const int n = *npass;
    const int nk_all = P.nkeys[b];
#pragma unroll
    for (int j = 0; j < GS_NB / 256; ++j) ((uint4*)hist)[j * 64 + lane] = make_uint4(0, 0, 0, 0);
    if (P.chain_status[b] != 0) {
        if (lane == 0) *npass = 0;
        return;
    }
    if (nk_all > P.ccap) {
        if (lane == 0) { *npass = 0; P.ncorners[b] = -1; }     // capacity: k_add_finish raises it
        return;
    }
    const int cs = P.cs, gw = P.gw, gh = P.gh, ncell = gw * gh;
    unsigned long long* gg =
        (unsigned long long*)(((uintptr_t)(P.ggrid + (int64_t)b * P.gstride) + 7) & ~(uintptr_t)7);
    for (int q = lane; q < ncell; q += 64) __hip_atomic_store(&gg[q], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    for (int q = lane; q < GS_HASH; q += 64) rhash[q] = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const uint64_t* sorted = P.sorted + (int64_t)b * P.sstride;
    float* out = P.corners + (int64_t)b * P.mcap * 2;
    int nacc = 0;
    const int limit = P.want;
    const uint64_t below = (1ull << lane) - 1ull;
    uint64_t knext = lane < n ? sorted[lane] : 0ull;
    for (int s0 = 0; s0 < n && nacc < limit; s0 += 64) {
        const int i = s0 + lane;
        bool tent = i < n;
        const uint32_t addr = (uint32_t)knext;
        knext = i + 64 < n ? sorted[i + 64] : 0ull;         // the next round's keys, in flight
        int y = (int)((float)addr * P.invW);
        y += ((uint32_t)(y + 1) * (uint32_t)P.W <= addr) ? 1 : 0;
        y -= ((uint32_t)y * (uint32_t)P.W > addr) ? 1 : 0;
        const int x = (int)(addr - (uint32_t)y * (uint32_t)P.W);
        const int xc = (int)__umulhi((uint32_t)x, P.cs_m), yc = (int)__umulhi((uint32_t)y, P.cs_m);
        const int x1 = max(xc - 1, 0), y1 = max(yc - 1, 0);
        const int x2 = min(xc + 1, gw - 1), y2 = min(yc + 1, gh - 1);
        // OpenCV's grid test against the corners accepted so far: the (up to) nine cells are
        // loaded together, then tested
        if (tent) {
            unsigned long long cv[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                const int yy = y1 + k / 3, xx = x1 + k % 3;
                cv[k] = (yy <= y2 && xx <= x2)
                            ? __hip_atomic_load(&gg[yy * gw + xx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
                            : 0ull;
            }
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                const int yy = y1 + k / 3, xx = x1 + k % 3;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t sl = (uint32_t)(cv[k] >> (16 * q)) & 0xFFFFu;
                    if (sl == 0) break;
                    const int ax = xx * cs + (int)((sl - 1) & 0xFFu), ay = yy * cs + (int)((sl - 1) >> 8);
                    const float ddx = (float)x - (float)ax, ddy = (float)y - (float)ay;
                    if ((double)(ddx * ddx + ddy * ddy) < P.md2) tent = false;
                }
            }
        }
        const uint64_t tmask = __ballot(tent);
        if (tmask == 0) continue;
        // conflicts with earlier candidates of this round: lanes register in a cell hash, each
        // reads the masks of its 3x3 neighbourhood and tests the (rare) earlier lanes exactly
        if (tent) {
            rxy[lane] = (uint32_t)x | ((uint32_t)y << 16);
            atomicOr((unsigned long long*)&rhash[(yc * gw + xc) & (GS_HASH - 1)], 1ull << lane);
        }
        wave_lds_sync();
        uint64_t conf = 0;
        if (tent) {
            uint64_t m = 0;
            for (int yy = y1; yy <= y2; ++yy)
                for (int xx = x1; xx <= x2; ++xx) m |= rhash[(yy * gw + xx) & (GS_HASH - 1)];
            m &= tmask & below;
            for (; m; m &= m - 1) {
                const int j = __builtin_ctzll(m);
                const uint32_t a = rxy[j];
                const int tx = (int)(a & 0xFFFF), ty = (int)(a >> 16);
                const int tcx = (int)__umulhi((uint32_t)tx, P.cs_m), tcy = (int)__umulhi((uint32_t)ty, P.cs_m);
                if (abs(tcx - xc) <= 1 && abs(tcy - yc) <= 1) {
                    const float ddx = (float)x - (float)tx, ddy = (float)y - (float)ty;
                    if ((double)(ddx * ddx + ddy * ddy) < P.md2) conf |= 1ull << j;
                }
            }
        }
        wave_lds_sync();
        if (tent) rhash[(yc * gw + xc) & (GS_HASH - 1)] = 0;
        // in-order resolution: a lane with conflicts is accepted iff none of its earlier
        // conflicting lanes is
        const uint64_t cm = __ballot(conf != 0);
        uint64_t amask = tmask & ~cm;
        for (uint64_t m = cm; m; m &= m - 1) {
            const int j = __builtin_ctzll(m);
            const uint64_t cj = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)conf, j) |
                                ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(conf >> 32), j) << 32);
            if ((cj & amask) == 0) amask |= 1ull << j;
        }
        // maxCorners: the first (limit - nacc) accepted lanes
        int nnew = __popcll(amask);
        if (nnew > limit - nacc) {
            uint64_t m = amask, keep = 0;
            for (int c = 0; c < limit - nacc; ++c) { const uint64_t lb = m & (~m + 1ull); keep |= lb; m ^= lb; }
            amask = keep;
            nnew = limit - nacc;
        }
        if ((amask >> lane) & 1ull) {
            const int idx = nacc + __popcll(amask & below);
            out[2 * idx] = (float)x;
            out[2 * idx + 1] = (float)y;
            // into the first free slot of its cell (two lanes of a round may share a cell); the
            // CAS returns before the wave goes on, so the next round's loads see it
            const unsigned long long code = 1ull + ((unsigned long long)(x - xc * cs) | ((unsigned long long)(y - yc * cs) << 8));
            unsigned long long* cp = &gg[yc * gw + xc];
            unsigned long long cur = __hip_atomic_load(cp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            for (;;) {
                int q = 0;
                while (q < 3 && ((cur >> (16 * q)) & 0xFFFFull)) ++q;
                const unsigned long long nv = cur | (code << (16 * q));
                if (__hip_atomic_compare_exchange_strong(cp, &cur, nv, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_WORKGROUP))
                    break;
            }
        }
        nacc += nnew;
        // one wave: its LDS operations and its returned atomics are complete in issue order; no
        // memory wait here (a fence would wait for the next round's key loads and the corner
        // stores every round)
        wave_lds_sync();
    }
    if (lane == 0) {
        P.ncorners[b] = nacc;
        P.nkeys[b] = n;
        *npass = 0;
    }
}

}  // namespace

// ======================================================================= host side
static inline bool hip_ok() { return hipGetLastError() == hipSuccess; }
#define VO_STREAM(s) ((hipStream_t)(s))

// GFTT selection form (vo_set_gftt_select): 0 = automatic, 1 = k_gftt_select, 2 = k_gsel_*
static int g_sel_mode = 0;
extern "C" int vo_set_gftt_select(int mode)
{
    if (mode < 0 || mode > 2) return VO_EARG;
    g_sel_mode = mode;
    return VO_OK;
}

extern "C" int vo_pyr_build(const vo_dims* d, const vo_state* s, int cur, const uint8_t* frames,
                            int64_t frame_stride, vo_stream_t stream)
{
    if (!d || !s || !frames || cur < 0 || cur > 1 || d->nlev < 1) return VO_EARG;
    // very few chains (the drop-in class's one): levels 0 and 1 in one launch (k_pyr01; one chain
    // 1,992-2,015 -> 2,029-2,049 frames/s eager).  At 32 chains per launch (the sequence job) the
    // fused kernel's 30 KB of LDS and byte-wise frame staging cost more than the launch saves
    // (29.4k -> 29.0k frames/s).  VO_PYR01=0 / 1 forces it off / on.
    static const int p01_env = [] { const char* e = getenv("VO_PYR01"); return e ? atoi(e) : -1; }();
    const bool fuse01 = d->nlev >= 2 && (p01_env >= 0 ? p01_env == 1 : d->B <= 8);
    if (fuse01) {
        PyrLevelArgs A0, A1;
        A0.src = frames; A0.sstride = frame_stride; A0.sw = A0.sh = A0.spitch = 0; A0.soff = 0;
        A1.src = frames; A1.sstride = frame_stride; A1.sw = d->lvl_w[0]; A1.sh = d->lvl_h[0]; A1.spitch = 0; A1.soff = 0;
        PyrLevelArgs* As[2] = {&A0, &A1};
        for (int l = 0; l < 2; ++l) {
            PyrLevelArgs& A = *As[l];
            A.pyr = s->pyr[cur]; A.pstride = d->pyr_stride;
            A.der = s->der[cur]; A.dstride = d->der_stride;
            A.w = d->lvl_w[l]; A.h = d->lvl_h[l]; A.pitch = d->lvl_pitch[l]; A.off = d->lvl_off[l];
            A.level = l;
            if (A.pitch % 64 || A.pitch < A.w + 2 * VO_BORDER) return VO_EARG;
        }
        const int pw0 = A0.w + 2 * VO_BORDER, ph0 = A0.h + 2 * VO_BORDER;
        const int pw1 = A1.w + 2 * VO_BORDER, ph1 = A1.h + 2 * VO_BORDER;
        const int tx0 = (pw0 + PT_W - 1) / PT_W, ty0 = (ph0 + PYR0_TH - 1) / PYR0_TH;
        const int tx1 = (pw1 + PT_W - 1) / PT_W, ty1 = (ph1 + PT_H - 1) / PT_H;
        dim3 g(tx0 > tx1 ? tx0 : tx1, ty0 + ty1, d->B);
        hipLaunchKernelGGL(k_pyr01, g, dim3(256), 0, VO_STREAM(stream), A0, A1, tx0, ty0, tx1);
    }
    // row-streaming single-wave levels (k_pyr_rows) unless VO_PYR_ROWS=0 (the tile kernels)
    static const int rows_env = [] { const char* e = getenv("VO_PYR_ROWS"); return e ? atoi(e) : 1; }();
    // levels 2.. of 9 to 64 chains in one launch (k_pyr_tail; VO_PYR_TAIL=0 / 1 forces it off /
    // on).  Rank 0 of the 8-GPU sequence plan (2 groups of 12 chains) 79.5-80.9k -> 83.0-83.9k
    // frames/s predicted; at one chain the per-level launches, with 48 waves a level instead of
    // 16, are faster (2,250 vs 2,185 frames/s; profiles/r5_pyr_tail_ab.jsonl)
    static const int tail_env = [] { const char* e = getenv("VO_PYR_TAIL"); return e ? atoi(e) : -1; }();
    const int ltail = 2;
    const bool tail = rows_env != 0 && d->nlev > ltail && d->nlev - ltail <= PYR_TAIL_MAX &&
                      (tail_env >= 0 ? tail_env == 1 : d->B > 8 && d->B <= 64);
    PyrTailArgs T;
    T.n = 0;
    if (tail) {
        T.n = d->nlev - ltail;
        for (int i = 0; i < T.n; ++i) {
            const int l = ltail + i;
            PyrLevelArgs& A = T.a[i];
            A.src = s->pyr[cur]; A.sstride = d->pyr_stride;
            A.sw = d->lvl_w[l - 1]; A.sh = d->lvl_h[l - 1]; A.spitch = d->lvl_pitch[l - 1]; A.soff = d->lvl_off[l - 1];
            A.pyr = s->pyr[cur]; A.pstride = d->pyr_stride;
            A.der = s->der[cur]; A.dstride = d->der_stride;
            A.w = d->lvl_w[l]; A.h = d->lvl_h[l]; A.pitch = d->lvl_pitch[l]; A.off = d->lvl_off[l];
            A.level = l;
            if (A.pitch % 64 || A.pitch < A.w + 2 * VO_BORDER) return VO_EARG;
            // about one item per wave of the 16-wave block
            const int pwa = (A.w + 2 * VO_BORDER + 3) & ~3, ns = (pwa + PR_STEP - 1) / PR_STEP;
            const int want = ns >= 16 ? 1 : 16 / ns;
            int R = (A.h + want - 1) / want;
            T.R[i] = R < 2 ? 2 : R;
        }
    }
    const int lend = tail ? ltail : d->nlev;
    for (int l = fuse01 ? 2 : 0; l < lend; ++l) {
        PyrLevelArgs A;
        if (l == 0) {
            A.src = frames; A.sstride = frame_stride; A.sw = A.sh = A.spitch = 0; A.soff = 0;
        } else {
            A.src = s->pyr[cur]; A.sstride = d->pyr_stride;
            A.sw = d->lvl_w[l - 1]; A.sh = d->lvl_h[l - 1]; A.spitch = d->lvl_pitch[l - 1]; A.soff = d->lvl_off[l - 1];
        }
        A.pyr = s->pyr[cur]; A.pstride = d->pyr_stride;
        A.der = s->der[cur]; A.dstride = d->der_stride;
        A.w = d->lvl_w[l]; A.h = d->lvl_h[l]; A.pitch = d->lvl_pitch[l]; A.off = d->lvl_off[l];
        A.level = l;
        const int pw = A.w + 2 * VO_BORDER, ph = A.h + 2 * VO_BORDER;
        if (A.pitch % 64 || A.pitch < pw) return VO_EARG;
        if (rows_env != 0) {
            // rows per wave: 16, fewer on small levels so that a launch still has >= 8k waves
            const int ns = ((pw + 3) / 4 * 4 + PR_STEP - 1) / PR_STEP;
            int R = 16;
            while (R > 4 && (int64_t)ns * ((A.h + R - 1) / R) * d->B < 8192) R >>= 1;
            dim3 g(ns, (A.h + R - 1) / R, d->B);
            if (l == 0) hipLaunchKernelGGL(k_pyr_rows<true>, g, dim3(64), 0, VO_STREAM(stream), A, R);
            else hipLaunchKernelGGL(k_pyr_rows<false>, g, dim3(64), 0, VO_STREAM(stream), A, R);
            continue;
        }
        // level 0 (frame bytes, small LDS): 32-row tiles, half the blocks; pyrDown levels: 16
        if (l == 0) {
            dim3 g((pw + PT_W - 1) / PT_W, (ph + PYR0_TH - 1) / PYR0_TH, d->B);
            hipLaunchKernelGGL((k_pyr_level<true, PYR0_TH>), g, dim3(256), 0, VO_STREAM(stream), A);
        } else {
            // tile rows of the pyrDown levels (VO_PYR_TH1 = 8 / 16 / 32 for experiments)
            static const int th1 = [] { const char* e = getenv("VO_PYR_TH1"); return e ? atoi(e) : PT_H; }();
            const int th = (th1 == 8 || th1 == 32) ? th1 : 16;
            dim3 g((pw + PT_W - 1) / PT_W, (ph + th - 1) / th, d->B);
            if (th == 8) hipLaunchKernelGGL((k_pyr_level<false, 8>), g, dim3(256), 0, VO_STREAM(stream), A);
            else if (th == 32) hipLaunchKernelGGL((k_pyr_level<false, 32>), g, dim3(256), 0, VO_STREAM(stream), A);
            else hipLaunchKernelGGL((k_pyr_level<false, 16>), g, dim3(256), 0, VO_STREAM(stream), A);
        }
    }
    if (tail) hipLaunchKernelGGL(k_pyr_tail, dim3(d->B), dim3(1024), 0, VO_STREAM(stream), T);
    return hip_ok() ? VO_OK : VO_EHIP;
}

extern "C" int vo_pyr_deriv(const vo_dims* d, const vo_state* s, int which, vo_stream_t stream)
{
    if (!d || !s || which < 0 || which > 1) return VO_EARG;
    for (int l = 0; l < d->nlev; ++l) {
        const int pw = d->lvl_w[l] + 2 * VO_BORDER, ph = d->lvl_h[l] + 2 * VO_BORDER;
        dim3 g((pw + 4 * 64 - 1) / (4 * 64), (ph + 3) / 4, d->B);
        hipLaunchKernelGGL(k_scharr, g, dim3(256), 0, VO_STREAM(stream), s->pyr[which], d->pyr_stride, s->der[which],
                           d->der_stride, d->lvl_w[l], d->lvl_h[l], d->lvl_pitch[l], d->lvl_off[l]);
    }
    return hip_ok() ? VO_OK : VO_EHIP;
}

static void fill_lk(LKParams& P, const vo_dims* d, const vo_opts* o, const vo_state* s, int prev)
{
    P.prev = s->pyr[prev];
    P.next = s->pyr[1 - prev];
    P.der = s->der[prev];
    P.pstride = d->pyr_stride;
    P.dstride = d->der_stride;
    P.L = d->nlev - 1;
    for (int l = 0; l < VO_MAX_LEVELS; ++l) {
        P.lw[l] = d->lvl_w[l];
        P.lh[l] = d->lvl_h[l];
        P.lpitch[l] = d->lvl_pitch[l];
        P.loff[l] = d->lvl_off[l];
    }
    P.win_w = o->win_w;
    P.win_h = o->win_h;
    int mc = o->crit_count;
    double eps = o->crit_eps;
    if (!(o->crit_type & 1)) mc = 30;
    else mc = mc < 0 ? 0 : (mc > 100 ? 100 : mc);
    if (!(o->crit_type & 2)) eps = 0.01;
    else eps = eps < 0 ? 0 : (eps > 10 ? 10 : eps);
    P.max_count = mc;
    P.eps2 = eps * eps;
    P.min_eig = (float)o->min_eig;
    // fl32(ddx^2 + ddy^2) (one rounded square, one fma) is within 2^-23 of the exact sum, plus
    // 2^-125 absolute near underflow: outside eps2 * (1 -+ 2^-20) it decides the double test
    // (eps2 >= 2^-100 keeps the absolute part far below the margin)
    if (P.eps2 >= 0x1p-100 && P.eps2 <= 0x1p100) {
        P.eps2_lo = nextafterf((float)(P.eps2 * (1. - 0x1p-20)), 0.f);
        P.eps2_hi = nextafterf((float)(P.eps2 * (1. + 0x1p-20)), INFINITY);
    } else {
        P.eps2_lo = -INFINITY;
        P.eps2_hi = INFINITY;
    }
}

static int launch_lk(const LKParams& P, int B, hipStream_t st)
{
    const int npx = P.win_w * P.win_h;
    if (P.win_w <= 2 || P.win_h <= 2 || npx > 64 * 16 || B < 1) return VO_EARG;
    // One wave per block (iteration counts differ wildly between points, so a wave's slot
    // must free as soon as its own points are done), 2048 blocks per chain.
    static const int nb_env = [] { const char* e = getenv("VO_LK_NB"); return e ? atoi(e) : 0; }();
    static const int xcd_env = [] { const char* e = getenv("VO_LK_XCD"); return e ? atoi(e) : 0; }();
    // 2048 blocks per chain: at ~1,900 points per C2 chain most waves carry one point, which
    // evens out the tail (headline 56.8k vs 56.1k frames/s with 1024, 56.7k with 4096)
    const int nb = nb_env > 0 ? nb_env : 2048;
    const int nblk = (B >= 8 ? ((B + 7) / 8) * 8 : B) * nb;
    // the LDS-staged 15x15 kernel reads whole dwords: it needs >= 64 bytes of slack after
    // the last pyramid level
    const int L = P.L;
    const int64_t pyr_end = P.loff[L] + (int64_t)(P.lh[L] + 2 * VO_BORDER) * P.lpitch[L];
    const bool staged15 = P.win_w == 15 && P.win_h == 15 && P.pstride >= pyr_end + 64;
    const size_t lds = 4 * (size_t)(P.win_w + 2 * LK_M) * (P.win_h + 2 * LK_M);
    if (lds > 60 * 1024) return VO_EARG;
    // 15x15 (every reference configuration, main.py:36,66,96): all levels in one launch, each
    // wave carrying its point from the coarsest level to level 0 in registers.  Other window
    // sizes (cv2.calcOpticalFlowPyrLK's default 21x21 on the cv2compat surface): k_lk, one
    // launch per level.
    if (staged15) {
        hipLaunchKernelGGL((k_lk_w<15, 15>), dim3(nblk), dim3(64), 0, st, P, L, 0, B, nb, xcd_env);
        return hip_ok() ? VO_OK : VO_EHIP;
    }
    for (int level = P.L; level >= 0; --level) {
        if (npx <= 256) hipLaunchKernelGGL(k_lk<4>, dim3(nblk), dim3(64), lds, st, P, level, B, nb);
        else hipLaunchKernelGGL(k_lk<16>, dim3(nblk), dim3(64), lds, st, P, level, B, nb);
    }
    return hip_ok() ? VO_OK : VO_EHIP;
}

extern "C" int vo_track(const vo_dims* d, const vo_opts* o, const vo_state* s, int prev, vo_stream_t stream)
{
    if (!d || !o || !s || prev < 0 || prev > 1) return VO_EARG;
    LKParams P;
    fill_lk(P, d, o, s, prev);
    P.p0 = s->lm_kp; P.n0 = s->nL; P.cap0 = d->ncap;
    P.p1 = s->c_kp; P.n1 = s->nC; P.cap1 = d->pcap; P.seg1_min = 1;   // :286 "if P > 1"
    P.chain_status = s->status;
    P.out = s->trk_pts; P.st = s->trk_st; P.err = s->trk_err; P.ocap = d->ncap + d->pcap;
    int rc = launch_lk(P, d->B, VO_STREAM(stream));
    if (rc) return rc;
    hipLaunchKernelGGL(k_track_compact, dim3(d->B), dim3(256), 0, VO_STREAM(stream), *d, *s);
    return hip_ok() ? VO_OK : VO_EHIP;
}

extern "C" int vo_track_lk(const vo_dims* d, const vo_opts* o, const vo_state* s, int prev, vo_stream_t stream)
{
    if (!d || !o || !s || prev < 0 || prev > 1) return VO_EARG;
    LKParams P;
    fill_lk(P, d, o, s, prev);
    P.p0 = s->lm_kp; P.n0 = s->nL; P.cap0 = d->ncap;
    P.p1 = s->c_kp; P.n1 = s->nC; P.cap1 = d->pcap; P.seg1_min = 1;   // :286 "if P > 1"
    P.chain_status = s->status;
    P.out = s->trk_pts; P.st = s->trk_st; P.err = s->trk_err; P.ocap = d->ncap + d->pcap;
    return launch_lk(P, d->B, VO_STREAM(stream));
}

extern "C" int vo_lk_points(const vo_dims* d, const vo_opts* o, const vo_state* s, int prev, const float* pts,
                            const int32_t* counts, int32_t cap, float* out_pts, uint8_t* out_status, float* out_err,
                            vo_stream_t stream)
{
    if (!d || !o || !s || !pts || !counts || !out_pts || !out_status) return VO_EARG;
    LKParams P;
    fill_lk(P, d, o, s, prev);
    P.p0 = pts; P.n0 = counts; P.cap0 = cap;
    P.p1 = nullptr; P.n1 = nullptr; P.cap1 = 0; P.seg1_min = 0;
    P.chain_status = nullptr;
    P.out = out_pts; P.st = out_status; P.err = out_err; P.ocap = cap;
    return launch_lk(P, d->B, VO_STREAM(stream));
}

#ifdef VO_LK_PROF
extern "C" int vo_lk_prof_read(long long* out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lkprof), sizeof g_lkprof) == hipSuccess ? VO_OK : VO_EHIP;
}
#endif

// eigen + NMS pass: the row-streaming k_eig3 for blockSize 3 / min-eigenvalue (every
// reference configuration), the tiled k_eignms otherwise (or with VO_EIG_GENERIC=1)
static void launch_eig(EigParams E, hipStream_t st)
{
    static const int generic = [] { const char* e = getenv("VO_EIG_GENERIC"); return e ? atoi(e) : 0; }();
    if (E.bs == 3 && !E.harris && !generic) {
        E.tiles_x = (E.W + E3_OUT - 1) / E3_OUT;
        E.tiles_y = (E.H + E3_TH - 1) / E3_TH;
        const int total = E.B * E.tiles_x * E.tiles_y;
        hipLaunchKernelGGL(k_eig3, dim3(((total + 7) / 8) * 8), dim3(64), 0, st, E);
        return;
    }
    const int total = E.B * E.tiles_x * E.tiles_y;
    hipLaunchKernelGGL(k_eignms, dim3(((total + 7) / 8) * 8), dim3(256), 0, st, E);
}

extern "C" int vo_gftt_eigmap(const vo_dims* d, const vo_opts* o, const vo_state* s, int cur, vo_stream_t stream)
{
    if (!d || !o || !s || cur < 0 || cur > 1) return VO_EARG;
    if (o->feature_block_size < 1 || o->feature_block_size > EIG_MAXBS) return VO_EARG;
    hipStream_t st = VO_STREAM(stream);
    if (hipMemsetAsync(s->eig_max, 0, sizeof(uint32_t) * d->B, st) != hipSuccess) return VO_EHIP;
    EigParams E;
    E.pyr = s->pyr[cur]; E.pstride = d->pyr_stride; E.W = d->W; E.H = d->H; E.pitch = d->lvl_pitch[0];
    E.off = d->lvl_off[0]; E.bs = o->feature_block_size; E.harris = o->feature_use_harris; E.harris_k = o->harris_k;
    E.eig_max = s->eig_max; E.keys = nullptr; E.nkeys = nullptr; E.ccap = 0;
    E.B = d->B; E.tiles_x = (d->W + EIG_TW - 1) / EIG_TW; E.tiles_y = (d->H + EIG_TH - 1) / EIG_TH;
    E.chain_status = nullptr;
    E.eig_out = s->eig;
    launch_eig(E, st);
    return hip_ok() ? VO_OK : VO_EHIP;
}

extern "C" int vo_gftt(const vo_dims* d, const vo_opts* o, const vo_state* s, int cur, vo_stream_t stream)
{
    if (!d || !o || !s || cur < 0 || cur > 1) return VO_EARG;
    if (o->feature_block_size < 1 || o->feature_block_size > EIG_MAXBS) return VO_EARG;
    hipStream_t st = VO_STREAM(stream);
    if (hipMemsetAsync(s->eig_max, 0, sizeof(uint32_t) * d->B, st) != hipSuccess) return VO_EHIP;
    if (hipMemsetAsync(s->gf_n, 0, sizeof(int32_t) * d->B, st) != hipSuccess) return VO_EHIP;
    EigParams E;
    E.pyr = s->pyr[cur]; E.pstride = d->pyr_stride; E.W = d->W; E.H = d->H; E.pitch = d->lvl_pitch[0];
    E.off = d->lvl_off[0]; E.bs = o->feature_block_size; E.harris = o->feature_use_harris; E.harris_k = o->harris_k;
    E.eig_max = s->eig_max; E.keys = s->gf_keys; E.nkeys = s->gf_n; E.ccap = d->ccap;
    E.B = d->B; E.tiles_x = (d->W + EIG_TW - 1) / EIG_TW; E.tiles_y = (d->H + EIG_TH - 1) / EIG_TH;
    E.chain_status = s->status;
    E.eig_out = nullptr;
    launch_eig(E, st);
    {
        // the split selection (k_gsel_*) where it applies: a minDistance grid of cells cvRound(md)
        // <= 255 wide (u64 cells of four corners: five never fit a cell of side cs - 1 <=
        // md - 0.5) that fits the eigen-map scratch, and 1 <= maxCorners <= the corner capacity
        // (no capacity truncation to report)
        const double md = o->feature_min_dist;
        const int cs = md >= 1 ? (int)lrint(md) : 0;
        const int gw = cs ? (d->W + cs - 1) / cs : 0, gh = cs ? (d->H + cs - 1) / cs : 0;
        const int64_t cells = (int64_t)gw * gh;
        const int want = o->feature_max_corners;
        const bool ok = s->gf_sort && cs >= 1 && cs <= 255 && cells * 8 + 4 <= (int64_t)4 * d->W * d->H && want >= 1 &&
                        want <= d->mcap && d->W <= 65535 && d->H <= 65535;
        static const int env = [] { const char* e = getenv("VO_SEL_SPLIT"); return e ? atoi(e) : -1; }();
        // automatic: the split form for more than 64 chains per launch, where the one-block
        // kernel waits for whole CUs beside the other stream group's LK flood (headline 384: the
        // GFTT stage 5.7 -> 1.9 ms; C5 128: 9.7k -> 10.2k frames/s); at 1-48 chains the GPU has
        // room for the fat block and its 512-1024 threads finish the walk sooner (one chain
        // 2,251 vs 2,213 frames/s; the 8-GPU slice of 2 x 12 chains 88.2k vs 82.7k predicted)
        const int mode = g_sel_mode ? g_sel_mode : (env >= 0 ? (env ? 2 : 1) : (d->B > 64 ? 2 : 1));
        if (ok && mode == 2) {
            SelSplitParams G;
            G.keys = s->gf_keys; G.nkeys = s->gf_n; G.eig_max = s->eig_max; G.quality = o->feature_quality_level;
            G.ccap = d->ccap; G.W = d->W; G.H = d->H; G.invW = 1.0f / (float)d->W;
            G.want = want; G.md2 = md * md; G.cs = cs; G.gw = gw; G.gh = gh;
            G.cs_m = (uint32_t)(((1ull << 32) + cs - 1) / cs);
            G.corners = s->corners; G.ncorners = s->nCorners; G.mcap = d->mcap;
            G.sorted = s->gf_sort; G.sstride = (int64_t)d->ccap + VO_GF_SORT_EXTRA;
            G.ggrid = s->eig; G.gstride = (int64_t)d->W * d->H;
            // waves per chain for the gate / scatter / rank: ~4k local maxima per wave at full
            // capacity (C2: 57, C5: 64); a wave with nothing left returns at once
            int wpc = d->ccap / 4096;
            G.wpc = wpc < 4 ? 4 : (wpc > 64 ? 64 : wpc);
            G.chain_status = s->status;
            const int nb = d->B * G.wpc;
            hipLaunchKernelGGL(k_gsel_gate, dim3(nb), dim3(64), 0, st, G);
            hipLaunchKernelGGL(k_gsel_scan, dim3(d->B), dim3(64), 0, st, G);
            hipLaunchKernelGGL(k_gsel_scatter, dim3(nb), dim3(64), 0, st, G);
            hipLaunchKernelGGL(k_gsel_rank, dim3(nb), dim3(64), 0, st, G);
            hipLaunchKernelGGL(k_gsel_walk, dim3(d->B), dim3(64), 0, st, G);
            return hip_ok() ? VO_OK : VO_EHIP;
        }
    }
    SelParams S;
    S.keys = s->gf_keys; S.nkeys = s->gf_n; S.ccap = d->ccap; S.W = d->W; S.H = d->H;
    S.eig_max = s->eig_max; S.quality = o->feature_quality_level;
    S.max_corners = o->feature_max_corners; S.min_dist = o->feature_min_dist;
    S.corners = s->corners; S.ncorners = s->nCorners; S.mcap = d->mcap; S.chain_status = s->status;
    S.gscratch = (uint32_t*)s->eig;      // L2 grid when the LDS grid is too small
    S.gstride = (int64_t)d->W * d->H;
    {
        // LDS sized to this configuration (page + corner cap + grid) instead of the maximum
        const double md = o->feature_min_dist;
        const int cs = md >= 1 ? (int)lrint(md) : 1;
        const int64_t cells = md >= 1 ? (int64_t)((d->W + cs - 1) / cs) * ((d->H + cs - 1) / cs) : 0;
        S.acc_lds = d->mcap < ACC_MAX ? d->mcap : ACC_MAX;
        S.grid_lds = cells <= GRID_LDS_CELLS ? (int)cells : 0;
        // grid + per-cell candidate lists in LDS when they fit, else in the eigen-map scratch
        // (after the conflict lists) for the same parallel walk, else the wave-serial L2 path
        if (16 * (size_t)PAGE + 4 * (size_t)S.acc_lds + 8 * (size_t)S.grid_lds > 150 * 1024) S.grid_lds = 0;
        static const int noglb = [] { const char* e = getenv("VO_SEL_SERIAL_L2"); return e ? atoi(e) : 0; }();
        S.grid_glb = !noglb && S.grid_lds == 0 && SEL_GG_OFF + 2 * cells <= S.gstride;
        const size_t lds = 16 * (size_t)PAGE + 4 * (size_t)S.acc_lds + 8 * (size_t)S.grid_lds;
        static const bool attr_ok =
            hipFuncSetAttribute((const void*)k_gftt_select<SEL_THREADS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                150 * 1024) == hipSuccess &&
            hipFuncSetAttribute((const void*)k_gftt_select<1024>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024) ==
                hipSuccess &&
            hipFuncSetAttribute((const void*)k_gftt_select<256>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024) ==
                hipSuccess;
        if (!attr_ok && lds > 64 * 1024) return VO_EHIP;
        // block size SEL_THREADS = 512, or VO_SEL_THREADS = 256 / 1024 (same result).  Headline
        // bench: 512 threads 56.2k frames/s, 1024 55.1k, 256 55.9k -- a select block holds its
        // wave slots while the other stream group's LK runs
        static const int nt_env = [] { const char* e = getenv("VO_SEL_THREADS"); return e ? atoi(e) : 0; }();
        // few chains (the GPU is mostly idle during the select): 1024 threads per chain
        const int nt_sel = nt_env ? nt_env : (d->B <= 128 ? 1024 : SEL_THREADS);
        if (nt_sel == 256) hipLaunchKernelGGL(k_gftt_select<256>, dim3(d->B), dim3(256), lds, st, S);
        else if (nt_sel == 1024) hipLaunchKernelGGL(k_gftt_select<1024>, dim3(d->B), dim3(1024), lds, st, S);
        else hipLaunchKernelGGL(k_gftt_select<SEL_THREADS>, dim3(d->B), dim3(SEL_THREADS), lds, st, S);
    }
    return hip_ok() ? VO_OK : VO_EHIP;
}
