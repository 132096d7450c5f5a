// SIFT (OpenCV 4.6 defaults) and brute-force 2-NN matching for gfx950
// (VisualOdometryPipeLine.py:35-36, :209-245).  SIFT stages: exact 2x upsample,
// separable Gaussian scale space (taps summed in a fixed order), DoG, 26-neighbour
// extrema (atomic candidate append -- order is irrelevant because keypoints are
// canonically sorted), per-candidate refinement + orientation histogram, LDS bitonic
// sort + dedupe (KeyPointsFilter::removeDuplicatedSorted), per-keypoint descriptor.
// Every float operation mirrors oracle/vo_oracle_sift.c.
//
// The matcher computes the query x train dot products with v_mfma_f32_32x32x16_bf16:
// SIFT descriptor entries are integers 0..255 (exact in bf16) and sums stay below 2^24,
// so distances are exact; the per-query top-2 scan keeps OpenCV's tie order.
#include "vo_dev.h"
#include "vo_crmath.h"

#include <stdlib.h>

#include <float.h>
#include <limits.h>
#include <math.h>
#include <string.h>

#define N_LAYERS 3
#define SIFT_IMG_BORDER 5
#define SIFT_MAX_INTERP_STEPS 5
#define SIFT_ORI_HIST_BINS 36
#define SIFT_ORI_SIG_FCTR 1.5f
#define SIFT_ORI_RADIUS (3 * SIFT_ORI_SIG_FCTR)
#define SIFT_ORI_PEAK_RATIO 0.8f
#define SIFT_DESCR_SCL_FCTR 3.f
#define SIFT_DESCR_MAG_THR 0.2f
#define SIFT_INT_DESCR_FCTR 512.f
#define KTAPS 32
#define EXPTAB_OFF (7 * KTAPS)

namespace {

// ------------------------------------------------------- exp32f / fastAtan2 (OpenCV)
#define EXPPOLY_32F_A0 .9670371139572337719125840413672004409288e-2

VO_DEV float exp32f(float x, const float* tab)
{
    const float A4 = (float)(1.000000000000002438532970795181890933776 / EXPPOLY_32F_A0);
    const float A3 = (float)(.6931471805521448196800669615864773144641 / EXPPOLY_32F_A0);
    const float A2 = (float)(.2402265109513301490103372422686535526573 / EXPPOLY_32F_A0);
    const float A1 = (float)(.5550339366753125211915322047004666939128e-1 / EXPPOLY_32F_A0);
    const float prescale = (float)(1.4426950408889634073599246810019 * (1 << 6));
    const float postscale = (float)(1. / (1 << 6));
    float x0 = x * prescale;
    int xi = __float2int_rn(x0);
    x0 = (x0 - (float)xi) * postscale;
    int t = (xi >> 6) + 127;
    t = !(t & ~255) ? t : (t < 0 ? 0 : 255);
    const float two = __int_as_float(t << 23);
    return two * tab[xi & 63] * ((((x0 + A1) * x0 + A2) * x0 + A3) * x0 + A4);
}

// a wave-uniform float (every lane holds the same value) in a scalar register
VO_DEV float uniform_f(float x) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x))); }

VO_DEV float fast_atan2(float y, float x)
{
    const float p1 = 0.9997878412794807f * (float)(180 / M_PI);
    const float p3 = -0.3258083974640975f * (float)(180 / M_PI);
    const float p5 = 0.1555786518463281f * (float)(180 / M_PI);
    const float p7 = -0.04432655554792128f * (float)(180 / M_PI);
    // OpenCV's two branches (|x| >= |y|: c = |y| / (|x| + eps), a = poly(c); else c = |x| / (|y| +
    // eps), a = 90 - poly(c)) as one division and one polynomial on selected operands: the same
    // operations per lane, but a wave whose lanes take both branches no longer runs both
    const float ax = fabsf(x), ay = fabsf(y);
    const bool xge = ax >= ay;
    const float c = (xge ? ay : ax) / ((xge ? ax : ay) + (float)DBL_EPSILON);
    const float c2 = c * c;
    const float pc = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    float a = xge ? pc : 90.f - pc;
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// ------------------------------------------------------- per-image views
// vo_sift_batch runs B images per launch: every buffer of vo_sift_buf holds B consecutive
// per-image blocks of the size vo_sift_plan reports; blockIdx.z is the image.
// Per-image base pointers of image z.  The kernels keep the vo_sift_buf kernel argument
// itself (offset tables indexed in kernarg memory) and address the data through these: a
// modified local copy of the whole struct would be dynamically indexed, i.e. live in scratch.
struct SiftImg {
    float* gauss;
    float* dog;
    int32_t* counters;
    int32_t* cand;
    float* kp;
    float* kp_out;
    float* desc;
    float* hist;
};
VO_DEV SiftImg sift_img(const vo_sift_buf& sb, int z)
{
    SiftImg p;
    p.gauss = sb.gauss + (int64_t)z * sb.gauss_floats;
    p.dog = sb.dog + (int64_t)z * sb.dog_floats;
    p.counters = sb.counters + 8 * z;
    p.cand = sb.cand + (int64_t)z * sb.cand_cap * 4;
    p.kp = sb.kp + (int64_t)z * sb.kp_cap * 8;
    p.kp_out = sb.kp_out + (int64_t)z * sb.kp_cap * 6;
    p.desc = sb.desc + (int64_t)z * sb.kp_cap * 128;
    p.hist = sb.hist + (int64_t)z * sb.kp_cap * 360;
    return p;
}

// ------------------------------------------------------- scale space
// 2x bilinear upsample (INTER_LINEAR, the reference's resize of the base image).  A block covers
// UP_ROWS output rows; a thread, one column of them (a one-row, 128-thread block per output row
// made 5.8 M blocks per 384-image launch, bound by block dispatch rather than by its 3 GB of
// stores).  The per-pixel arithmetic is unchanged.
#define UP_ROWS 8
__global__ void __launch_bounds__(256) k_upsample(const uint8_t* __restrict__ img, int64_t img_stride, int w, int h,
                                                  float* __restrict__ dst, int64_t dst_stride)
{
    const int dx = blockIdx.x * blockDim.x + threadIdx.x;
    const int dw = 2 * w, dh = 2 * h;
    if (dx >= dw) return;
    img += blockIdx.z * img_stride;
    dst += blockIdx.z * dst_stride;
    float fx = (float)((dx + 0.5) * 0.5 - 0.5);
    int sx = (int)floorf(fx);
    fx -= sx;
    if (sx < 0) { fx = 0; sx = 0; }
    if (sx >= w - 1) { fx = 0; sx = w - 1; }
    const int sx1 = sx + 1 < w ? sx + 1 : w - 1;
    const int dy0 = blockIdx.y * UP_ROWS;
    for (int dy = dy0; dy < dy0 + UP_ROWS && dy < dh; ++dy) {
        float fy = (float)((dy + 0.5) * 0.5 - 0.5);
        int sy = (int)floorf(fy);
        fy -= sy;
        if (sy < 0) { fy = 0; sy = 0; }
        if (sy >= h - 1) { fy = 0; sy = h - 1; }
        const int sy1 = sy + 1 < h ? sy + 1 : h - 1;
        const uint8_t* r0 = img + (int64_t)sy * w;
        const uint8_t* r1 = img + (int64_t)sy1 * w;
        const float v0 = (float)r0[sx] * (1.f - fx) + (float)r0[sx1] * fx;
        const float v1 = (float)r1[sx] * (1.f - fx) + (float)r1[sx1] * fx;
        dst[(int64_t)dy * dw + dx] = v0 * (1.f - fy) + v1 * fy;
    }
}

// Separable Gaussian (BORDER_REFLECT_101) of one 64 x 32 output tile per block, both
// passes through LDS: the source tile with its reflected halo is read from HBM once, the
// row pass fills an LDS tile of (32 + 2r) rows, the column pass writes the output -- and,
// when `dog` is given, the difference of Gaussians out - src at the same pixel (the next
// DoG layer, D_i = G_{i+1} - G_i), so the DoG never re-reads the scale space.  Taps are
// summed k = 0..n-1 in both passes, exactly as the two-pass form and the oracle do.
#define BT_W 64
#define BT_H 32
#define BT_R 13                  // largest radius: ksize 27
__global__ void __launch_bounds__(256) k_blur_tile(const float* __restrict__ src, int64_t src_stride,
                                                   float* __restrict__ dst, int64_t dst_stride,
                                                   float* __restrict__ dog, int64_t dog_stride, int w, int h,
                                                   const float* __restrict__ kern, int n)
{
    // LDS sized by the host for this kernel's radius (blur_lds): more blocks per CU for the
    // small kernels
    extern __shared__ float s_dyn[];
    __shared__ float s_k[2 * BT_R + 1];
    const int tid = threadIdx.x;
    const int r = n >> 1;
    float* s_src = s_dyn;
    // source row stride odd (cols + 1): the row pass's lanes read at 4-float steps from four
    // rows, which are then spread over all LDS banks
    const int sst = BT_W + 2 * r + 1;
    float* s_row = s_dyn + (BT_H + 2 * r) * sst;
    const int x0 = blockIdx.x * BT_W, y0 = blockIdx.y * BT_H;
    src += blockIdx.z * src_stride;
    const bool wdst = dst != nullptr;                  // null: the DoG alone (top layer)
    dst += blockIdx.z * dst_stride;
    if (tid < n) s_k[tid] = kern[tid];
    const int rows = BT_H + 2 * r, cols = BT_W + 2 * r;
    // staging: 64 lanes along a row, the four waves on rows w, w+4, ... (reflection computed per
    // row / column, no division per element).  Fixed trip counts, unrolled: every load of the
    // tile is in flight before the first LDS store (a load-store loop waited one memory round
    // trip per trip)
    {
        constexpr int NR = (BT_H + 2 * BT_R + 3) / 4, NC = (BT_W + 2 * BT_R + 63) / 64;
        const int lx = tid & 63, wy = tid >> 6;
        int xo[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) xo[c] = refl101(x0 - r + min(lx + 64 * c, cols - 1), w);
        float v[NR][NC];
#pragma unroll
        for (int j = 0; j < NR; ++j) {
            const int ty = min(wy + 4 * j, rows - 1);
            const float* srow = src + (int64_t)refl101(y0 - r + ty, h) * w;
#pragma unroll
            for (int c = 0; c < NC; ++c) v[j][c] = srow[xo[c]];
        }
#pragma unroll
        for (int j = 0; j < NR; ++j) {
            const int ty = wy + 4 * j;
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const int tx = lx + 64 * c;
                if (ty < rows && tx < cols) s_src[ty * sst + tx] = v[j][c];
            }
        }
    }
    __syncthreads();
    // row pass: four adjacent outputs per thread share one sliding window of n + 3 reads; each
    // output still sums its taps k = 0..n-1 in order
    for (int i = tid; i < rows * (BT_W / 4); i += 256) {
        const int ty = i >> 4, tx = (i & 15) * 4;
        const float* sp = s_src + ty * sst + tx;
        float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
        float v0 = sp[0], v1 = sp[1], v2 = sp[2];
        for (int k = 0; k < n; ++k) {
            const float v3 = sp[k + 3], kk = s_k[k];
            a0 += kk * v0; a1 += kk * v1; a2 += kk * v2; a3 += kk * v3;
            v0 = v1; v1 = v2; v2 = v3;
        }
        *reinterpret_cast<float4*>(s_row + ty * BT_W + tx) = make_float4(a0, a1, a2, a3);
    }
    __syncthreads();
    // column pass: four rows per thread (rows q, q + 8, q + 16, q + 24 would not share reads;
    // adjacent rows do)
    {
        const int tx = tid & 63, ty = (tid >> 6) * 8;
        const int gx = x0 + tx;
        for (int half = 0; half < 2; ++half) {
            const int tyh = ty + 4 * half;
            const float* sp = s_row + tyh * BT_W + tx;
            float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
            float v0 = sp[0], v1 = sp[BT_W], v2 = sp[2 * BT_W];
            for (int k = 0; k < n; ++k) {
                const float v3 = sp[(k + 3) * BT_W], kk = s_k[k];
                a0 += kk * v0; a1 += kk * v1; a2 += kk * v2; a3 += kk * v3;
                v0 = v1; v1 = v2; v2 = v3;
            }
            const float acc[4] = {a0, a1, a2, a3};
    #pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int gy = y0 + tyh + j;
                if (gy >= h || gx >= w) continue;
                if (wdst) dst[(int64_t)gy * w + gx] = acc[j];
                if (dog) dog[blockIdx.z * dog_stride + (int64_t)gy * w + gx] = acc[j] - s_src[(tyh + j + r) * sst + tx + r];
            }
        }
    }
}

// k_blur_tile for a compile-time kernel size N (the SIFT sizes 11, 13, 17, 21, 27), same
// tile, same staging, same tap order -- on packed FP32 (v_pk_mul_f32 / v_pk_add_f32: two
// independent IEEE operations per lane, rounded exactly as the scalar pair):
//  * taps in scalar registers (uniform loads of `kern`), no per-tap LDS read;
//  * row pass: a thread sums two rows x four columns, the pair of rows in one packed register
//    ({row y, row y+1} of each source column), N + 3 reads per row;
//  * column pass: a thread sums two columns x four rows, the column pair read as one 8-byte
//    LDS load per source row.
// One packed multiply + one packed add per tap per two outputs (the scalar form: two each).
typedef float vf2 __attribute__((ext_vector_type(2)));
template <int N>
__global__ void __launch_bounds__(256) k_blur_tile_n(const float* __restrict__ src, int64_t src_stride,
                                                     float* __restrict__ dst, int64_t dst_stride,
                                                     float* __restrict__ dog, int64_t dog_stride, int w, int h,
                                                     const float* __restrict__ kern)
{
    constexpr int r = N >> 1;
    constexpr int rows = BT_H + 2 * r, cols = BT_W + 2 * r, sst = cols + 1;
    static_assert(r <= BT_R && rows % 2 == 0, "k_blur_tile_n tile");
    __shared__ float s_src[rows * sst];
    __shared__ __attribute__((aligned(16))) float s_row[rows * BT_W];
    const int tid = threadIdx.x;
    const int x0 = blockIdx.x * BT_W, y0 = blockIdx.y * BT_H;
    src += blockIdx.z * src_stride;
    const bool wdst = dst != nullptr;                  // null: the DoG alone (top layer)
    dst += blockIdx.z * dst_stride;
    float kk[N];
#pragma unroll
    for (int k = 0; k < N; ++k) kk[k] = kern[k];
    {
        constexpr int NR = (rows + 3) / 4, NC = (cols + 63) / 64;
        const int lx = tid & 63, wy = tid >> 6;
        int xo[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) xo[c] = refl101(x0 - r + min(lx + 64 * c, cols - 1), w);
        float v[NR][NC];
#pragma unroll
        for (int j = 0; j < NR; ++j) {
            const int ty = min(wy + 4 * j, rows - 1);
            const float* srow = src + (int64_t)refl101(y0 - r + ty, h) * w;
#pragma unroll
            for (int c = 0; c < NC; ++c) v[j][c] = srow[xo[c]];
        }
#pragma unroll
        for (int j = 0; j < NR; ++j) {
            const int ty = wy + 4 * j;
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const int tx = lx + 64 * c;
                if (ty < rows && tx < cols) s_src[ty * sst + tx] = v[j][c];
            }
        }
    }
    __syncthreads();
    // row pass: item = rows (2 q, 2 q + 1) x columns 4 c .. 4 c + 3
    for (int i = tid; i < (rows / 2) * (BT_W / 4); i += 256) {
        const int ty = 2 * (i >> 4), tx = (i & 15) * 4;
        const float* sp = s_src + ty * sst + tx;
        vf2 v[N + 3];
#pragma unroll
        for (int m = 0; m < N + 3; ++m) v[m] = vf2{sp[m], sp[sst + m]};
        vf2 a0 = {0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0;
#pragma unroll
        for (int k = 0; k < N; ++k) {
            const vf2 kv = {kk[k], kk[k]};
            a0 = a0 + kv * v[k]; a1 = a1 + kv * v[k + 1]; a2 = a2 + kv * v[k + 2]; a3 = a3 + kv * v[k + 3];
        }
        *reinterpret_cast<float4*>(s_row + ty * BT_W + tx) = make_float4(a0.x, a1.x, a2.x, a3.x);
        *reinterpret_cast<float4*>(s_row + (ty + 1) * BT_W + tx) = make_float4(a0.y, a1.y, a2.y, a3.y);
    }
    __syncthreads();
    // column pass: columns (2 c, 2 c + 1) x rows 4 g .. 4 g + 3
    {
        const int tx = 2 * (tid & 31), ty = (tid >> 5) * 4;
        const float* sp = s_row + ty * BT_W + tx;
        vf2 v[N + 3];
#pragma unroll
        for (int m = 0; m < N + 3; ++m) v[m] = *reinterpret_cast<const vf2*>(sp + m * BT_W);
        vf2 a[4] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
        for (int k = 0; k < N; ++k) {
            const vf2 kv = {kk[k], kk[k]};
#pragma unroll
            for (int j = 0; j < 4; ++j) a[j] = a[j] + kv * v[k + j];
        }
        const int gx = x0 + tx;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int gy = y0 + ty + j;
            if (gy >= h) continue;
            const float* cs = s_src + (ty + j + r) * sst + tx + r;
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                if (gx + e >= w) continue;
                const float o = e ? a[j].y : a[j].x;
                if (wdst) dst[(int64_t)gy * w + gx + e] = o;
                if (dog) dog[blockIdx.z * dog_stride + (int64_t)gy * w + gx + e] = o - cs[e];
            }
        }
    }
}

__global__ void k_nn_down(const float* __restrict__ src, int sw, int sh, float* __restrict__ dst, int dw, int dh,
                          int64_t stride)
{
    const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= dw) return;
    src += blockIdx.z * stride;
    dst += blockIdx.z * stride;
    const double ifx = 1. / ((double)dw / sw), ify = 1. / ((double)dh / sh);
    int sy = (int)floor(y * ify);
    if (sy > sh - 1) sy = sh - 1;
    int sx = (int)floor(x * ifx);
    if (sx > sw - 1) sx = sw - 1;
    dst[(int64_t)y * dw + x] = src[(int64_t)sy * sw + sx];
}

// All three extremum layers of one octave from one LDS tile: 64 x 16 interior pixels per
// block, the five DoG layers of the octave with a 1-pixel halo staged once; each pixel that
// passes the threshold is compared with the max / min of its 3x3x3 neighbourhood (separable:
// 3-wide row max / min per layer and row, then 3 rows x 3 layers; no early exit -- the
// per-pixel loop with an exit at the first failing neighbour was a chain of dependent global
// loads).  The test is findScaleSpaceExtrema's:
// val > 0 && val >= every neighbour, or val < 0 && val <= every neighbour (the centre itself is
// one of the 27, which changes nothing).  Candidates are appended with one atomic per wave; the
// list order is irrelevant (keypoints are sorted canonically).
#define EX_W 64
#define EX_H 16
#define EX_LCAP 1024                      // candidates per block held in LDS (more: flagged)
__global__ void __launch_bounds__(256) k_extrema_t(vo_sift_buf sb, int o)
{
    const SiftImg im = sift_img(sb, blockIdx.z);
    __shared__ float t[N_LAYERS + 2][EX_H + 2][EX_W + 2];
    __shared__ int2 s_list[EX_LCAP];
    __shared__ int s_n, s_base;
    const int w = sb.oct_w[o], h = sb.oct_h[o];
    const int x0 = SIFT_IMG_BORDER + blockIdx.x * EX_W, y0 = SIFT_IMG_BORDER + blockIdx.y * EX_H;
    const int tid = threadIdx.x;
    if (tid == 0) s_n = 0;
    const float* dog0 = im.dog + sb.dog_off[o * (N_LAYERS + 2)];
    const int64_t plane = (int64_t)w * h;               // the octave's DoG layers are contiguous
    // every load of the tile in flight before the first LDS store (fixed, unrolled trip counts;
    // clamped addresses, zeros written outside the octave).  By rows: the four waves take rows
    // wy, wy + 4, ... of every layer, the 64 lanes columns 0..63 and lanes 0, 1 columns 64, 65 --
    // row / column arithmetic only (a flat element index cost two divisions per element)
    constexpr int TR = EX_H + 2, TC = EX_W + 2, NJ = (TR + 3) / 4;
    static_assert(TC == 66, "k_extrema_t staging: 64 + 2 columns");
    const __amdgpu_buffer_rsrc_t rdog =
        __builtin_amdgcn_make_buffer_rsrc((void*)dog0, (short)0, (int)(4 * (N_LAYERS + 2) * plane), 0x00020000);
    const int lx = tid & 63, wy = tid >> 6;
    const int gx0 = min(x0 - 1 + lx, w - 1), gx1 = min(x0 - 1 + 64 + (lx & 1), w - 1);
    float v0[N_LAYERS + 2][NJ], v1[N_LAYERS + 2][NJ];
#pragma unroll
    for (int l = 0; l < N_LAYERS + 2; ++l)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int ty = min(wy + 4 * j, TR - 1);
            const int row = l * (int)plane + min(y0 - 1 + ty, h - 1) * w;
            // buffer loads: 32-bit offsets, one VGPR per load
            v0[l][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rdog, 4 * (row + gx0), 0, 0));
            v1[l][j] = lx < 2 ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rdog, 4 * (row + gx1), 0, 0))
                              : 0.f;
        }
#pragma unroll
    for (int l = 0; l < N_LAYERS + 2; ++l)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int ty = wy + 4 * j;
            if (ty < TR) {
                const bool rin = y0 - 1 + ty < h;
                t[l][ty][lx] = (rin && x0 - 1 + lx < w) ? v0[l][j] : 0.f;
                if (lx < 2) t[l][ty][64 + lx] = (rin && x0 - 1 + 64 + lx < w) ? v1[l][j] : 0.f;
            }
        }
    __syncthreads();
    const float threshold = (float)floor(0.5 * 0.04 / N_LAYERS * 255 * 1);
    const int tx = tid & (EX_W - 1), ty0 = (tid >> 6) * (EX_H / 4);
    const int c = x0 + tx;
    const int lane = tid & 63;
    // a thread's four pixels are one column, rows ty0..ty0+3: the 3-wide row max / min of the six
    // tile rows under them, for all five layers, is read once (18 LDS reads per layer) and each
    // pixel's 27-neighbourhood max / min is the max / min of 9 of these
    constexpr int R = EX_H / 4 + 2;
    float hx[N_LAYERS + 2][R], hn[N_LAYERS + 2][R], ctr[N_LAYERS + 2][EX_H / 4];
    // layer l's row max / min are formed right before they are first needed (layer l - 1's
    // pixels), so at most three layers of them are live (fully unrolled)
#pragma unroll
    for (int l = 0; l < N_LAYERS + 2; ++l) {
#pragma unroll
        for (int rr = 0; rr < R; ++rr) {
            const float a0 = t[l][ty0 + rr][tx], a1 = t[l][ty0 + rr][tx + 1], a2 = t[l][ty0 + rr][tx + 2];
            hx[l][rr] = fmaxf(fmaxf(a0, a1), a2);
            hn[l][rr] = fminf(fminf(a0, a1), a2);
            if (rr >= 1 && rr <= EX_H / 4) ctr[l][rr - 1] = a1;
        }
        const int layer = l - 1;
        if (layer < 1) continue;
#pragma unroll
        for (int k = 0; k < EX_H / 4; ++k) {
            const int r = y0 + ty0 + k;
            const float val = ctr[layer][k];
            bool ext = c < w - SIFT_IMG_BORDER && r < h - SIFT_IMG_BORDER && fabsf(val) > threshold;
            float mx = val, mn = val;
#pragma unroll
            for (int dz = -1; dz <= 1; ++dz)
#pragma unroll
                for (int dy = 0; dy < 3; ++dy) {
                    mx = fmaxf(mx, hx[layer + dz][k + dy]);
                    mn = fminf(mn, hn[layer + dz][k + dy]);
                }
            ext = ext && (val > 0 ? val >= mx : val <= mn);
            const uint64_t m = __ballot(ext);
            if (m == 0) continue;
            // block-local list first (LDS atomic per wave): one global atomic per block at the
            // end -- a global atomic per wave on the image's one counter serialised in L2
            const int leader = __ffsll((unsigned long long)m) - 1;
            int base = 0;
            if (lane == leader) base = atomicAdd(&s_n, __popcll(m));
            base = __shfl(base, leader, 64);
            if (!ext) continue;
            const int q = base + __popcll(m & ((1ull << lane) - 1ull));
            if (q < EX_LCAP) s_list[q] = make_int2(layer, (r << 16) | c);
        }
    }
    __syncthreads();
    const int nl = s_n;
    if (nl == 0) return;
    if (tid == 0) s_base = atomicAdd(&im.counters[0], nl);
    __syncthreads();
    const int gbase = s_base;
    for (int i = tid; i < nl; i += 256) {
        const int q = gbase + i;
        if (i >= EX_LCAP || q >= sb.cand_cap) { im.counters[3] = 1; continue; }   // capacity: flagged
        const int2 e = s_list[i];
        im.cand[4 * q] = o; im.cand[4 * q + 1] = e.x; im.cand[4 * q + 2] = e.y >> 16; im.cand[4 * q + 3] = e.y & 0xFFFF;
    }
}

// ------------------------------------------------------- keypoints
#define DAT(base, w, r, c) ((base)[(int64_t)(r) * (w) + (c)])

VO_DEV void lu3_solve(float A[9], float b[3], float X[3])
{
    const float eps = FLT_EPSILON * 10;
    for (int i = 0; i < 3; ++i) {
        int k = i;
        for (int j = i + 1; j < 3; ++j) if (fabsf(A[j * 3 + i]) > fabsf(A[k * 3 + i])) k = j;
        if (fabsf(A[k * 3 + i]) < eps) { X[0] = X[1] = X[2] = 0; return; }
        if (k != i) {
            for (int j = i; j < 3; ++j) { float t = A[i * 3 + j]; A[i * 3 + j] = A[k * 3 + j]; A[k * 3 + j] = t; }
            float t = b[i]; b[i] = b[k]; b[k] = t;
        }
        float d = -1 / A[i * 3 + i];
        for (int j = i + 1; j < 3; ++j) {
            float alpha = A[j * 3 + i] * d;
            for (int kk = i + 1; kk < 3; ++kk) A[j * 3 + kk] += alpha * A[i * 3 + kk];
            b[j] += alpha * b[i];
        }
        A[i * 3 + i] = -d;
    }
    for (int i = 2; i >= 0; --i) {
        float s = b[i];
        for (int kk = i + 1; kk < 3; ++kk) s -= A[i * 3 + kk] * b[kk];
        b[i] = s * A[i * 3 + i];
    }
    X[0] = b[0]; X[1] = b[1]; X[2] = b[2];
}

struct KP { float x, y, size, angle, response; int octave; };

VO_DEV bool adjust_local_extrema(const vo_sift_buf& sb, const float* dogs, KP& kpt, int octv, int& layer, int& r, int& c, float sigma)
{
    const float contrastThreshold = 0.04f, edgeThreshold = 10.f;
    const float img_scale = 1.f / (255 * 1);
    const float deriv_scale = img_scale * 0.5f;
    const float second_deriv_scale = img_scale;
    const float cross_deriv_scale = img_scale * 0.25f;
    const int w = sb.oct_w[octv], h = sb.oct_h[octv];
    float xi = 0, xr = 0, xc = 0, contr = 0;
    int i = 0;
    for (; i < SIFT_MAX_INTERP_STEPS; ++i) {
        const int idx = octv * (N_LAYERS + 2) + layer;
        const float* img = dogs + sb.dog_off[idx];
        const float* prev = dogs + sb.dog_off[idx - 1];
        const float* next = dogs + sb.dog_off[idx + 1];
        float dD[3] = {(DAT(img, w, r, c + 1) - DAT(img, w, r, c - 1)) * deriv_scale,
                       (DAT(img, w, r + 1, c) - DAT(img, w, r - 1, c)) * deriv_scale,
                       (DAT(next, w, r, c) - DAT(prev, w, r, c)) * deriv_scale};
        float v2 = DAT(img, w, r, c) * 2;
        float dxx = (DAT(img, w, r, c + 1) + DAT(img, w, r, c - 1) - v2) * second_deriv_scale;
        float dyy = (DAT(img, w, r + 1, c) + DAT(img, w, r - 1, c) - v2) * second_deriv_scale;
        float dss = (DAT(next, w, r, c) + DAT(prev, w, r, c) - v2) * second_deriv_scale;
        float dxy = (DAT(img, w, r + 1, c + 1) - DAT(img, w, r + 1, c - 1) - DAT(img, w, r - 1, c + 1) +
                     DAT(img, w, r - 1, c - 1)) * cross_deriv_scale;
        float dxs = (DAT(next, w, r, c + 1) - DAT(next, w, r, c - 1) - DAT(prev, w, r, c + 1) +
                     DAT(prev, w, r, c - 1)) * cross_deriv_scale;
        float dys = (DAT(next, w, r + 1, c) - DAT(next, w, r - 1, c) - DAT(prev, w, r + 1, c) +
                     DAT(prev, w, r - 1, c)) * cross_deriv_scale;
        float H[9] = {dxx, dxy, dxs, dxy, dyy, dys, dxs, dys, dss};
        float X[3];
        lu3_solve(H, dD, X);
        xi = -X[2]; xr = -X[1]; xc = -X[0];
        if (fabsf(xi) < 0.5f && fabsf(xr) < 0.5f && fabsf(xc) < 0.5f) break;
        if (fabsf(xi) > (float)(INT_MAX / 3) || fabsf(xr) > (float)(INT_MAX / 3) || fabsf(xc) > (float)(INT_MAX / 3))
            return false;
        c += __float2int_rn(xc);
        r += __float2int_rn(xr);
        layer += __float2int_rn(xi);
        if (layer < 1 || layer > N_LAYERS || c < SIFT_IMG_BORDER || c >= w - SIFT_IMG_BORDER || r < SIFT_IMG_BORDER ||
            r >= h - SIFT_IMG_BORDER)
            return false;
    }
    if (i >= SIFT_MAX_INTERP_STEPS) return false;
    {
        const int idx = octv * (N_LAYERS + 2) + layer;
        const float* img = dogs + sb.dog_off[idx];
        const float* prev = dogs + sb.dog_off[idx - 1];
        const float* next = dogs + sb.dog_off[idx + 1];
        float dD[3] = {(DAT(img, w, r, c + 1) - DAT(img, w, r, c - 1)) * deriv_scale,
                       (DAT(img, w, r + 1, c) - DAT(img, w, r - 1, c)) * deriv_scale,
                       (DAT(next, w, r, c) - DAT(prev, w, r, c)) * deriv_scale};
        float t = dD[0] * xc + dD[1] * xr + dD[2] * xi;
        contr = DAT(img, w, r, c) * img_scale + t * 0.5f;
        if (fabsf(contr) * N_LAYERS < contrastThreshold) return false;
        float v2 = DAT(img, w, r, c) * 2.f;
        float dxx = (DAT(img, w, r, c + 1) + DAT(img, w, r, c - 1) - v2) * second_deriv_scale;
        float dyy = (DAT(img, w, r + 1, c) + DAT(img, w, r - 1, c) - v2) * second_deriv_scale;
        float dxy = (DAT(img, w, r + 1, c + 1) - DAT(img, w, r + 1, c - 1) - DAT(img, w, r - 1, c + 1) +
                     DAT(img, w, r - 1, c - 1)) * cross_deriv_scale;
        float tr = dxx + dyy;
        float det = dxx * dyy - dxy * dxy;
        if (det <= 0 || tr * tr * edgeThreshold >= (edgeThreshold + 1) * (edgeThreshold + 1) * det) return false;
    }
    kpt.x = ((float)c + xc) * (float)(1 << octv);
    kpt.y = ((float)r + xr) * (float)(1 << octv);
    kpt.octave = octv + (layer << 8) + ((int)rint((xi + 0.5) * 255) << 16);
    kpt.size = sigma * (float)vcr_exp2((double)(((float)layer + xi) / N_LAYERS)) * (float)(1 << octv) * 2;
    kpt.response = fabsf(contr);
    return true;
}

// Keypoint refinement and orientation in two stages:
//  k_sift_refine  adjustLocalExtrema per candidate (one thread each) -> refined records in
//                 the hist scratch (12 floats each), count in counters[4];
//  k_sift_ori     calcOrientationHist + peak interpolation with one WAVE per refined keypoint:
//                 lanes compute gradient / weight / bin of 64 window positions at a time (raster
//                 order), the 36 bins are owned by lanes 0..35 and each lane adds, in pixel order,
//                 the values that land in its bin -- the serial accumulation order, so the
//                 histogram, its smoothing, the peaks and the emitted keypoints are identical.
//                 Keypoints are appended with atomics; k_sift_sort_dedupe orders them.
#define SIFT_REC 12
__global__ void __launch_bounds__(128) k_sift_refine(vo_sift_buf sb)
{
    const SiftImg im = sift_img(sb, blockIdx.z);
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int nc = min(im.counters[0], sb.cand_cap);
    if (blockIdx.x * blockDim.x >= nc) return;
    int o = 0, r1 = 0, c1 = 0, layer = 0;
    KP kpt;
    bool ok = false;
    if (k < nc) {
        o = im.cand[4 * k];
        layer = im.cand[4 * k + 1];
        r1 = im.cand[4 * k + 2];
        c1 = im.cand[4 * k + 3];
        ok = adjust_local_extrema(sb, im.dog, kpt, o, layer, r1, c1, 1.6f);
    }
    // one atomic per wave (record order is irrelevant: keypoints are canonically sorted)
    const uint64_t m = __ballot(ok);
    if (m == 0) return;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((unsigned long long)m) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(&im.counters[4], __popcll(m));
    base = __shfl(base, leader, 64);
    if (!ok) return;
    const int rec_cap = (int)(((int64_t)sb.kp_cap * 360) / SIFT_REC);
    const int q = base + __popcll(m & ((1ull << lane) - 1ull));
    if (q >= rec_cap) { im.counters[3] = 1; return; }
    float* rec = im.hist + (int64_t)SIFT_REC * q;
    rec[0] = kpt.x; rec[1] = kpt.y; rec[2] = kpt.size; rec[3] = kpt.response;
    rec[4] = __int_as_float(kpt.octave); rec[5] = __int_as_float(o); rec[6] = __int_as_float(layer);
    rec[7] = __int_as_float(r1); rec[8] = __int_as_float(c1);
}

__global__ void __launch_bounds__(256) k_sift_ori(vo_sift_buf sb)
{
    const SiftImg im = sift_img(sb, blockIdx.z);
    __shared__ int4 pb_s4[4][18];
    __shared__ float4 pv_s4[4][16];
    __shared__ float th_s[4][SIFT_ORI_HIST_BINS + 4];
    __shared__ float hs_s[4][SIFT_ORI_HIST_BINS];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int rec_cap = (int)(((int64_t)sb.kp_cap * 360) / SIFT_REC);
    const int n_rec = min(im.counters[4], rec_cap);
    for (int q = blockIdx.x * 4 + w; q < n_rec; q += gridDim.x * 4) {   // wave-uniform loop
        int* pcnt = reinterpret_cast<int*>(pb_s4[w]);      // per bin: its pixels in the chunk
        int* poff = pcnt + 36;                              // per bin: its first slot
        float* pval = reinterpret_cast<float*>(pv_s4[w]);  // the chunk's values sorted by bin
        const float* rec = im.hist + (int64_t)SIFT_REC * q;
        // wave-uniform record fields in scalar registers (scalar loop control below)
        const float kx = rec[0], ky = rec[1], ksize = uniform_f(rec[2]), kresp = rec[3];
        const int koct = __float_as_int(rec[4]);
        const int o = __builtin_amdgcn_readfirstlane(__float_as_int(rec[5]));
        const int layer = __builtin_amdgcn_readfirstlane(__float_as_int(rec[6]));
        const int py = __builtin_amdgcn_readfirstlane(__float_as_int(rec[7]));
        const int px = __builtin_amdgcn_readfirstlane(__float_as_int(rec[8]));
        const float* tab = sb.consts + EXPTAB_OFF;
        const float scl_octv = ksize * 0.5f / (float)(1 << o);
        const float* img = im.gauss + sb.gauss_off[o * (N_LAYERS + 3) + layer];
        const int wd = sb.oct_w[o], ht = sb.oct_h[o];
        const int radius = __float2int_rn(SIFT_ORI_RADIUS * scl_octv);
        const float sigma = SIFT_ORI_SIG_FCTR * scl_octv;
        const int n = SIFT_ORI_HIST_BINS;
        const float expf_scale = -1.f / (2.f * sigma * sigma);
        const int side = 2 * radius + 1, total = side * side;
        const float inv_side = 1.f / (float)side;
        float th = 0.f;                                   // temphist[lane] for lane < 36
        for (int base = 0; base < total; base += 64) {
            const int pos = base + lane;
            bool valid = false;
            int bin = 0;
            float val = 0.f;
            if (pos < total) {
                // pos / side from the float reciprocal: exact (pos < 2^20; margin 0.5 / side)
                const int ii = (int)(((float)pos + 0.5f) * inv_side);
                const int i = ii - radius, j = pos - ii * side - radius;
                const int y = py + i, x = px + j;
                valid = y > 0 && y < ht - 1 && x > 0 && x < wd - 1;
                if (valid) {
                    const float dx = DAT(img, wd, y, x + 1) - DAT(img, wd, y, x - 1);
                    const float dy = DAT(img, wd, y - 1, x) - DAT(img, wd, y + 1, x);
                    const float wt = exp32f((float)(i * i + j * j) * expf_scale, tab);
                    const float ori = fast_atan2(dy, dx);
                    const float mag = sqrtf(dx * dx + dy * dy);
                    bin = __float2int_rn((n / 360.f) * ori);
                    if (bin >= n) bin -= n;
                    if (bin < 0) bin += n;
                    val = wt * mag;
                }
            }
            // Each bin's pixels must reach th in lane (= the serial raster) order.  The chunk's
            // valid pixels are sorted by bin, stably: a pixel's slot is the start of its bin
            // (an exclusive scan of the per-bin counts) plus its rank among the pixels of its bin
            // in lower lanes.  `eq` = the lanes holding my bin, from six bit-sliced ballots of the
            // 6-bit bin (invalid lanes hold bin 0 and are masked out by `m`).  Lane b then adds
            // its bin's pixels slot by slot: the same additions, in the same order, as the
            // pixel-by-pixel walk, in max-per-bin rounds instead of one pass per four pixels.
            const uint64_t m = __ballot(valid);
            uint32_t eq_lo = (uint32_t)m, eq_hi = (uint32_t)(m >> 32);
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                const uint32_t mine = (uint32_t)(-((bin >> k) & 1));      // ~0 if my bit k is set
                const uint64_t bk = __ballot(mine != 0u);
                eq_lo &= ~((uint32_t)bk ^ mine);
                eq_hi &= ~((uint32_t)(bk >> 32) ^ mine);
            }
            const int rank = (int)__builtin_amdgcn_mbcnt_hi(eq_hi, __builtin_amdgcn_mbcnt_lo(eq_lo, 0u));
            const int cnt_p = __popc(eq_lo) + __popc(eq_hi);
            if (lane < n) pcnt[lane] = 0;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (valid) pcnt[bin] = cnt_p;                   // every pixel of a bin writes the same
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const int c = lane < n ? pcnt[lane] : 0;        // pixels of bin `lane`
            int incl = c;                                   // inclusive scan over the lanes
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const int y = __shfl_up(incl, d, 64);
                if (lane >= d) incl += y;
            }
            const int off = incl - c;                       // first slot of bin `lane`
            if (lane < n) poff[lane] = off;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (valid) pval[poff[bin] + rank] = val;        // slots 0 .. popc(m) - 1
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            for (int k = 0; __ballot(k < c) != 0ull; ++k)
                if (k < c) th += pval[off + k];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        float* t2 = th_s[w];                              // temphist[-2 .. n+1] at t2[0 .. n+3]
        if (lane < n) t2[2 + lane] = th;
        if (lane == n - 1) t2[1] = th;                    // temphist[-1] = temphist[n-1]
        if (lane == n - 2) t2[0] = th;                    // temphist[-2] = temphist[n-2]
        if (lane == 0) t2[n + 2] = th;                    // temphist[n] = temphist[0]
        if (lane == 1) t2[n + 3] = th;                    // temphist[n+1] = temphist[1]
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        float hv = -FLT_MAX;
        if (lane < n) {
            const float* t = t2 + 2 + lane;
            hv = (t[-2] + t[2]) * (1.f / 16.f) + (t[-1] + t[1]) * (4.f / 16.f) + t[0] * (6.f / 16.f);
            hs_s[w][lane] = hv;
        }
        float omax = hv;
    #pragma unroll
        for (int off = 32; off >= 1; off >>= 1) omax = fmaxf(omax, __shfl_xor(omax, off, 64));
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const float mag_thr = (float)(omax * SIFT_ORI_PEAK_RATIO);
        if (lane < n) {
            const float* hist = hs_s[w];
            const int j = lane;
            const int l = j > 0 ? j - 1 : n - 1;
            const int r2 = j < n - 1 ? j + 1 : 0;
            if (hist[j] > hist[l] && hist[j] > hist[r2] && hist[j] >= mag_thr) {
                float bin = j + 0.5f * (hist[l] - hist[r2]) / (hist[l] - 2 * hist[j] + hist[r2]);
                bin = bin < 0 ? n + bin : bin >= n ? bin - n : bin;
                float angle = 360.f - (float)((360.f / n) * bin);
                if (fabsf(angle - 360.f) < FLT_EPSILON) angle = 0.f;
                const int qo = atomicAdd(&im.counters[1], 1);
                if (qo < sb.kp_cap) {
                    float* out = im.kp + 8 * (int64_t)qo;
                    out[0] = kx; out[1] = ky; out[2] = ksize; out[3] = angle; out[4] = kresp;
                    out[5] = __int_as_float(koct); out[6] = 0.f; out[7] = 0.f;
                } else {
                    im.counters[3] = 1;
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// KeyPoint12_LessThan: x asc, y asc, size desc, angle asc, response desc, octave desc
VO_DEV bool kp_less(const float* a, const float* b)
{
    if (a[0] != b[0]) return a[0] < b[0];
    if (a[1] != b[1]) return a[1] < b[1];
    if (a[2] != b[2]) return a[2] > b[2];
    if (a[3] != b[3]) return a[3] < b[3];
    if (a[4] != b[4]) return a[4] > b[4];
    const int oa = __float_as_int(a[5]), ob = __float_as_int(b[5]);
    if (oa != ob) return oa > ob;
    return false;
}

// keypoint indices as 16-bit LDS entries: 32,768 raw keypoints per image in 64 KB
#define SORT_N 32768
#define SORT_PAD 0xFFFFu
__global__ void __launch_bounds__(1024) k_sift_sort_dedupe(vo_sift_buf sb)
{
    const SiftImg im = sift_img(sb, blockIdx.z);
    __shared__ uint16_t idx[SORT_N];
    __shared__ int lds[16];
    const int tid = threadIdx.x;
    const int n = min(im.counters[1], sb.kp_cap);
    if (n > SORT_N) { if (tid == 0) im.counters[3] = 1; }
    const int nn = n < SORT_N ? n : SORT_N;
    int P = 1;
    while (P < nn) P <<= 1;
    for (int i = tid; i < P; i += blockDim.x) idx[i] = i < nn ? (uint16_t)i : (uint16_t)SORT_PAD;
    __syncthreads();
    for (int size = 2; size <= P; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = tid; i < P / 2; i += blockDim.x) {
                const int lo = 2 * i - (i & (stride - 1));
                const int hi = lo + stride;
                const bool asc = ((lo & size) == 0);
                const unsigned a = idx[lo], c = idx[hi];
                // "a > c" in kp_less order, padding sorts last
                bool gt;
                if (a == SORT_PAD) gt = c != SORT_PAD;
                else if (c == SORT_PAD) gt = false;
                else gt = kp_less(im.kp + 8 * (int64_t)c, im.kp + 8 * (int64_t)a);
                if (gt == asc) { idx[lo] = (uint16_t)c; idx[hi] = (uint16_t)a; }
            }
            __syncthreads();
        }
    }
    int out = 0;
    for (int base = 0; base < nn; base += blockDim.x) {
        const int i = base + tid;
        bool keep = false;
        const float* k = nullptr;
        if (i < nn) {
            k = im.kp + 8 * (int64_t)idx[i];
            keep = true;
            if (i > 0) {
                const float* p = im.kp + 8 * (int64_t)idx[i - 1];
                keep = (k[0] != p[0] || k[1] != p[1] || k[2] != p[2] || k[3] != p[3]);
            }
        }
        int tot;
        const int pos = out + block_scan_flag(keep, lds, &tot);
        if (keep) {
            float* o = im.kp_out + 6 * (int64_t)pos;
            int oct = __float_as_int(k[5]);
            oct = (oct & ~255) | ((oct - 1) & 255);                      // firstOctave = -1
            o[0] = k[0] * 0.5f; o[1] = k[1] * 0.5f; o[2] = k[2] * 0.5f; o[3] = k[3]; o[4] = k[4];
            o[5] = (float)oct;
        }
        out += tot;
    }
    if (tid == 0) im.counters[2] = out;
}

// ------------------------------------------------------- KeyPointsFilter::retainBest
// SIFT_create(nfeatures) (BASELINE C5: "SIFT capped at the best 8192"): after
// removeDuplicatedSorted, retainBest(keypoints, nfeatures) (features2d/src/keypoint.cpp) =
// std::nth_element(KeypointResponseGreater) on the n-th position, then std::partition of the
// rest by response >= that boundary response, then resize.  The kept keypoints stay in the
// order libstdc++'s algorithms leave them (the BF query order downstream); the oracle restates
// them step for step (oracle/vo_oracle_sift.c) and tests/test_retain_best.py pins that against
// the real std::nth_element.  The firstOctave scaling in k_sift_sort_dedupe does not touch the
// response, so selecting after it is the same.
//
// Block-parallel form of every Hoare round of __introselect: the scan pointer i stops at the
// k-th "left stopper" (!(r > pivot)) and j at the k-th "right stopper" (!(pivot > r)) of the
// range in the ORIGINAL order, as long as they have not crossed (the elements a swap moves
// are stoppers for the other pointer, so nothing in between changes).  A round therefore
// compacts both stopper lists with ordered block scans, counts K = #{k : L_k < R_k} (monotone),
// swaps the K pairs at once, and cuts at min(L_K, R_{K-1}).  std::partition's bidirectional
// loop is the same pairing with the stoppers !(r >= amb) / (r >= amb).  The median-of-3 pivot
// move, the final insertion sort of <= 3 records and the depth-limit __heap_select fallback
// (adversarial inputs only) run on one thread, like libstdc++.  Records (response bits, index)
// live in the image's candidate buffer, free after k_sift_refine.
#define RB_T 1024
VO_DEV bool rb_gt(int2 a, int2 b) { return __int_as_float(a.x) > __int_as_float(b.x); }
VO_DEV void rb_swap(int2* a, int2* b) { const int2 t = *a; *a = *b; *b = t; }

VO_DEV void rb_move_median_to_first(int2* result, int2* a, int2* b, int2* c)
{
    if (rb_gt(*a, *b)) {
        if (rb_gt(*b, *c)) rb_swap(result, b);
        else if (rb_gt(*a, *c)) rb_swap(result, c);
        else rb_swap(result, a);
    } else if (rb_gt(*a, *c)) rb_swap(result, a);
    else if (rb_gt(*b, *c)) rb_swap(result, c);
    else rb_swap(result, b);
}

VO_DEV void rb_adjust_heap(int2* first, int hole, int len, int2 value)
{
    const int top = hole;
    int second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (rb_gt(first[second], first[second - 1])) second--;
        first[hole] = first[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        first[hole] = first[second - 1];
        hole = second - 1;
    }
    int parent = (hole - 1) / 2;                                   // __push_heap
    while (hole > top && rb_gt(first[parent], value)) {
        first[hole] = first[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    first[hole] = value;
}

VO_DEV void rb_heap_select(int2* first, int2* middle, int2* last)
{
    const int len = (int)(middle - first);
    if (len >= 2)
        for (int parent = (len - 2) / 2;; --parent) {
            rb_adjust_heap(first, parent, len, first[parent]);
            if (parent == 0) break;
        }
    for (int2* i = middle; i < last; ++i)
        if (rb_gt(*i, *first)) {
            const int2 v = *i;
            *i = *first;
            rb_adjust_heap(first, 0, len, v);
        }
}

VO_DEV void rb_insertion_sort(int2* first, int2* last)
{
    if (first == last) return;
    for (int2* i = first + 1; i != last; ++i) {
        const int2 v = *i;
        if (rb_gt(v, *first)) {
            for (int2* p = i; p != first; --p) *p = *(p - 1);
            *first = v;
        } else {
            int2* hole = i;
            int2* nx = i - 1;
            while (rb_gt(v, *nx)) { *hole = *nx; hole = nx; --nx; }
            *hole = v;
        }
    }
}

// Stopper lists of the pair-swap partition of rec[a, b): LP ascending positions with
// lstop(r), RP descending positions with rstop(r); returns K = number of pairs
// (LP[k], RP[k]) with LP[k] < RP[k], after swapping them.  rsent >= 0 appends that position
// to RP (the unguarded scan's pivot sentinel).  Every thread returns the same values.
template <class LS, class RS>
VO_DEV int rb_pairs(int2* rec, int a, int b, LS lstop, RS rstop, int rsent, int* LP, int* RP, int* lds, int* nl_out,
                    int* nr_out)
{
    const int tid = threadIdx.x;
    int nL = 0, nR = 0;
    for (int base = a; base < b; base += RB_T) {
        const int p = base + tid;
        const bool f = p < b && lstop(__int_as_float(rec[p].x));
        int tot;
        const int pos = block_scan_flag(f, lds, &tot);
        if (f) LP[nL + pos] = p;
        nL += tot;
    }
    for (int base = 0; base < b - a; base += RB_T) {
        const int q = b - 1 - base - tid;
        const bool f = q >= a && rstop(__int_as_float(rec[q].x));
        int tot;
        const int pos = block_scan_flag(f, lds, &tot);
        if (f) RP[nR + pos] = q;
        nR += tot;
    }
    if (rsent >= 0) {
        if (tid == 0) RP[nR] = rsent;
        ++nR;
    }
    __syncthreads();
    // K: the pairs are ordered (LP ascending, RP descending), so LP[k] < RP[k] holds for a prefix
    const int m = nL < nR ? nL : nR;
    int cnt = 0;
    for (int k = tid; k < m; k += RB_T) cnt += LP[k] < RP[k] ? 1 : 0;
    int K;
    block_scan_i32(cnt, lds, &K);
    for (int k = tid; k < K; k += RB_T) rb_swap(&rec[LP[k]], &rec[RP[k]]);
    __syncthreads();
    *nl_out = nL;
    *nr_out = nR;
    return K;
}

__global__ void __launch_bounds__(RB_T) k_sift_retain_best(vo_sift_buf sb)
{
    const SiftImg im = sift_img(sb, blockIdx.z);
    const int n = im.counters[2];
    const int P = sb.nfeatures;
    if (P <= 0 || n <= P) return;                                  // retainBest keeps everything
    __shared__ int lds[16];
    __shared__ int bc[2];
    const int tid = threadIdx.x;
    int2* rec = reinterpret_cast<int2*>(im.cand);
    int* LP = im.cand + 2 * n;
    int* RP = LP + n + 1;
    for (int i = tid; i < n; i += RB_T) rec[i] = make_int2(__float_as_int(im.kp_out[6 * (int64_t)i + 4]), i);
    __syncthreads();
    // std::nth_element(first, first + P - 1, last): __introselect with depth 2 * __lg(n)
    const int nth = P - 1;
    int first = 0, last = n, depth = 2 * (31 - __clz(n));
    bool heap = false;
    while (last - first > 3) {
        if (depth == 0) {
            if (tid == 0) {
                rb_heap_select(rec + first, rec + nth + 1, rec + last);
                rb_swap(rec + first, rec + nth);
            }
            heap = true;
            break;
        }
        --depth;
        if (tid == 0)                                              // __unguarded_partition_pivot
            rb_move_median_to_first(rec + first, rec + first + 1, rec + first + (last - first) / 2, rec + last - 1);
        __syncthreads();
        const float pv = __int_as_float(rec[first].x);
        int nL, nR;
        const int K = rb_pairs(
            rec, first + 1, last, [pv](float r) { return !(r > pv); }, [pv](float r) { return !(pv > r); }, first, LP,
            RP, lds, &nL, &nR);
        if (tid == 0) {
            // i stops at L_{K+1}, or at R_K (it now holds a left stopper) if that comes first
            int cut = K < nL ? LP[K] : last;
            if (K > 0 && RP[K - 1] < cut) cut = RP[K - 1];
            bc[0] = cut;
        }
        __syncthreads();
        const int cut = bc[0];
        __syncthreads();
        if (cut <= nth) first = cut;
        else last = cut;
    }
    if (!heap && tid == 0) rb_insertion_sort(rec + first, rec + last);
    __syncthreads();
    // std::partition(first + P, last, response >= kp[P - 1].response), then resize
    const float amb = __int_as_float(rec[nth].x);
    int nL, nR;
    rb_pairs(
        rec, P, n, [amb](float r) { return !(r >= amb); }, [amb](float r) { return r >= amb; }, -1, LP, RP, lds, &nL,
        &nR);
    const int kept = n - nL;                                       // every non-stopper is kept
    // gather the kept rows in their new order (through the raw keypoint buffer, free now)
    float* tmp = im.kp;
    for (int i = tid; i < kept * 6; i += RB_T) tmp[i] = im.kp_out[6 * (int64_t)rec[i / 6].y + i % 6];
    __syncthreads();
    for (int i = tid; i < kept * 6; i += RB_T) im.kp_out[i] = tmp[i];
    if (tid == 0) im.counters[2] = kept;
}

// k_sift_desc_w: calcSIFTDescriptor with one WAVE per keypoint and the same arithmetic, in
// the same order, as the C restatement (oracle/vo_oracle_sift.c).
//  * window positions are processed 64 at a time in raster order: each lane computes one
//    position's gradient, weight, bins and its eight trilinear contributions (the per-pixel
//    math, in parallel); the valid ones are compacted into LDS in raster order;
//  * the histogram (360 bins) lives in LDS.  The eight bins a pixel touches
//    (idx + {0, 1, 10, 11, 60, 61, 70, 71}) are distinct, so eight lanes update them with one
//    read-add-write; pixels follow in raster order (lds_rmw_add4_lanes), so each bin receives
//    its additions in exactly the serial order;
//  * the 128-entry normalisation sums stay sequential (lane 0), clamps / scaling run per lane;
//  * 8 waves per SIMD: the 128-float descriptor row reuses the contribution buffer (19.7 KB of
//    LDS per 4-wave block) and VGPRs are capped at 64 -- the walk is LDS-latency bound, so the
//    extra waves pay for the few per-keypoint spills (batch-64 KITTI desc -15 %).
// Histogram update of the descriptor walk: hist[p] += v0, v1, v2, v3 in that order for the
// lanes in `lanes` (wave-uniform), i.e. a run of up to four pixels with the same eight bins --
// one read, the four adds in pixel order (missing pixels add +0, which leaves a bin unchanged:
// every contribution and every partial sum is >= +0), one write.  Written as asm with exec
// narrowed to the run's lanes: straight-line code, no branch per run.  A wave's LDS operations
// execute in issue order, so the next run's read sees this write.  (ds_add_f32 on the same
// lanes is exact too but measured 4x slower: LDS float atomics run at a fraction of the
// read/write rate.)
VO_DEV void lds_rmw_add4_lanes(float* p, float v0, float v1, float v2, float v3, uint64_t lanes)
{
    const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)p;
    uint64_t save;
    float h;
    asm volatile("s_mov_b64 %0, exec\n\ts_and_b64 exec, exec, %7\n\tds_read_b32 %1, %2\n\ts_waitcnt lgkmcnt(0)\n\t"
                 "v_add_f32 %1, %1, %3\n\tv_add_f32 %1, %1, %4\n\tv_add_f32 %1, %1, %5\n\tv_add_f32 %1, %1, %6\n\t"
                 "ds_write_b32 %2, %1\n\ts_mov_b64 exec, %0"
                 : "=&s"(save), "=&v"(h)
                 : "v"(a), "v"(v0), "v"(v1), "v"(v2), "v"(v3), "s"(lanes)
                 : "memory", "scc");        // s_and_b64 writes SCC
}

// The eight read-add-writes of one group of sub-runs (lanes 8 j .. 8 j + 7 serve sub-run j), in
// sub-run order, as one asm block: exec is set to the group's lanes by one 32-bit SALU op per
// step (steps 0-3 in exec_lo, 4-7 in exec_hi) instead of saving / masking / restoring it around
// every step (k_sift_desc_w shares the CU's one scalar unit with its VALU work; SALU-heavy code
// waits on it).  Same LDS operations in the same order as eight lds_rmw_add4_lanes calls.
VO_DEV void lds_rmw_add4_walk8(float* p, float v0, float v1, float v2, float v3, uint64_t am)
{
    const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)p;
    const uint32_t am_lo = (uint32_t)am, am_hi = (uint32_t)(am >> 32);
    uint64_t save;
    float h;
#define VO_RMW4 "ds_read_b32 %1, %2\n\ts_waitcnt lgkmcnt(0)\n\tv_add_f32 %1, %1, %3\n\tv_add_f32 %1, %1, %4\n\t" \
                "v_add_f32 %1, %1, %5\n\tv_add_f32 %1, %1, %6\n\tds_write_b32 %2, %1\n\t"
    asm volatile("s_mov_b64 %0, exec\n\t"
                 "s_mov_b32 exec_hi, 0\n\ts_and_b32 exec_lo, %7, 0xff\n\t" VO_RMW4
                 "s_and_b32 exec_lo, %7, 0xff00\n\t" VO_RMW4
                 "s_and_b32 exec_lo, %7, 0xff0000\n\t" VO_RMW4
                 "s_and_b32 exec_lo, %7, 0xff000000\n\t" VO_RMW4
                 "s_mov_b32 exec_lo, 0\n\ts_and_b32 exec_hi, %8, 0xff\n\t" VO_RMW4
                 "s_and_b32 exec_hi, %8, 0xff00\n\t" VO_RMW4
                 "s_and_b32 exec_hi, %8, 0xff0000\n\t" VO_RMW4
                 "s_and_b32 exec_hi, %8, 0xff000000\n\t" VO_RMW4
                 "s_mov_b64 exec, %0"
                 : "=&s"(save), "=&v"(h)
                 : "v"(a), "v"(v0), "v"(v1), "v"(v2), "v"(v3), "s"(am_lo), "s"(am_hi)
                 : "memory", "scc");        // s_and_b32 writes SCC
#undef VO_RMW4
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) k_sift_desc_w(vo_sift_buf sb)
{
    const SiftImg im = sift_img(sb, blockIdx.z);
    __shared__ int4 pidx_s4[4][16];
    int (*pidx_s)[64] = reinterpret_cast<int (*)[64]>(pidx_s4);
    // contributions k-major with a 72-float stride: the pixel phase's stores (one per k, 64
    // lanes) and the walk's loads (lane 8j + k reads pixel g + j's k-th) are conflict-free
    __shared__ float pval_s[4][8 * 72];
    __shared__ float hist_s[4][384];
    __shared__ float red_s[4][2];
    __shared__ uint32_t ring_s[4][128];
    __shared__ int slist_s[4][64];
    // exp32f's 64-entry table in LDS (a gather per pixel: no global round trip)
    __shared__ float tab_s[64];
    if (threadIdx.x < 64) tab_s[threadIdx.x] = sb.consts[EXPTAB_OFF + threadIdx.x];
    __syncthreads();
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n_kp = im.counters[2];
    // cos / sin of every keypoint this wave will describe, one keypoint per lane: the
    // correctly rounded double-double evaluations (vo_crmath.h) are long serial FP64 chains, so
    // they run once per wave instead of once per keypoint
    const int qs = gridDim.x * 4, qf = blockIdx.x * 4 + w;
    float lane_cos = 0.f, lane_sin = 0.f;
    {
        const int ql = qf + lane * qs;
        if (ql < n_kp) {
            float angle = 360.f - im.kp_out[6 * (int64_t)ql + 3];
            if (fabsf(angle - 360.f) < FLT_EPSILON) angle = 0.f;
            lane_cos = (float)vcr_cos((double)(angle * (float)(M_PI / 180)));
            lane_sin = (float)vcr_sin((double)(angle * (float)(M_PI / 180)));
        }
    }
    int qi = 0;
    for (int q = qf; q < n_kp; q += qs, ++qi) {                           // wave-uniform loop
        int* pidx = pidx_s[w];
        float* pval = pval_s[w];
        float* hist = hist_s[w];
        float* dsl = pval_s[w];       // the walk's contributions are dead once it ends
        uint32_t* ring = ring_s[w];
        int* slist = slist_s[w];
        const float* tab = tab_s;
        // the keypoint's fields are wave-uniform: read them into scalar registers, so that every
        // quantity derived from them (window radius, trip counts, ring state) is known uniform and
        // the loops below branch on scalars instead of exec masks
        const float* kp = im.kp_out + 6 * (int64_t)q;
        const int kpo = __builtin_amdgcn_readfirstlane((int)kp[5]);
        int octave = kpo & 255, layer = (kpo >> 8) & 255;
        octave = octave < 128 ? octave : (-128 | octave);
        const float scale = octave >= 0 ? 1.f / (1 << octave) : (float)(1 << -octave);
        const float size = uniform_f(kp[2]) * scale;
        const float ptx = uniform_f(kp[0]) * scale, pty = uniform_f(kp[1]) * scale;
        const int oi = octave + 1;
        const float* img = im.gauss + sb.gauss_off[oi * (N_LAYERS + 3) + layer];
        const int cols = sb.oct_w[oi], rows = sb.oct_h[oi];
        float angle = 360.f - uniform_f(kp[3]);
        if (fabsf(angle - 360.f) < FLT_EPSILON) angle = 0.f;
        const float ori = angle, scl = size * 0.5f;
        const int d = 4, n = 8;
        const int ptix = __float2int_rn(ptx), ptiy = __float2int_rn(pty);
        float cos_t, sin_t;
        if (qi < 64) {
            cos_t = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(lane_cos), qi));
            sin_t = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(lane_sin), qi));
        } else {
            cos_t = (float)vcr_cos((double)(ori * (float)(M_PI / 180)));
            sin_t = (float)vcr_sin((double)(ori * (float)(M_PI / 180)));
        }
        const float bins_per_rad = n / 360.f;
        const float exp_scale = -1.f / (d * d * 0.5f);
        const float hist_width = SIFT_DESCR_SCL_FCTR * scl;
        int radius = __float2int_rn(hist_width * 1.4142135623730951f * (d + 1) * 0.5f);
        const int rmax = (int)sqrt(((double)cols) * cols + ((double)rows) * rows);
        if (radius > rmax) radius = rmax;
        cos_t /= hist_width;
        sin_t /= hist_width;
        const int side = 2 * radius + 1;
        const int total = side * side;
        for (int t = lane; t < 384; t += 64) hist[t] = 0.f;
        // Window positions in raster order, 64 at a time: the valid ones (inside the rotated
        // descriptor square and the image) are appended, in order, to a 128-entry ring; every 64
        // pending positions form one dense chunk whose per-pixel math runs on all 64 lanes, and
        // whose contributions are then walked into the histogram.  Chunks stay in raster order.
        const float inv_side = 1.f / (float)side;
        int head = 0, pend = 0;                                      // wave-uniform ring state
        for (int base = 0; base < total; base += 64) {
            const int pos = base + lane;
            // pos / side from the float reciprocal: exact (pos < 2^20; margin 0.5 / side)
            const int ii = (int)(((float)pos + 0.5f) * inv_side);
            const int i = ii - radius, j = pos - ii * side - radius;
            const float c_rot = j * cos_t - i * sin_t;
            const float r_rot = j * sin_t + i * cos_t;
            const float rbin = r_rot + d / 2 - 0.5f;
            const float cbin = c_rot + d / 2 - 0.5f;
            const int r = ptiy + i, c = ptix + j;
            // every term evaluated (no short circuit: one flat mask computation, no exec juggling)
            const bool valid = (pos < total) & (rbin > -1) & (rbin < d) & (cbin > -1) & (cbin < d) & (r > 0) &
                               (r < rows - 1) & (c > 0) & (c < cols - 1);
            const uint64_t m = __ballot(valid);
            if (valid)
                ring[(head + pend + __popcll(m & ((1ull << lane) - 1ull))) & 127] =
                    (uint32_t)(uint16_t)i | ((uint32_t)(uint16_t)j << 16);
            pend += __popcll(m);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const bool last = base + 64 >= total;
            while (pend >= 64 || (last && pend > 0)) {
                const int take = pend < 64 ? pend : 64;
                if (lane < take) {
                    const uint32_t e = ring[(head + lane) & 127];
                    const int pi = (int)(int16_t)(e & 0xFFFF), pj = (int)(int16_t)(e >> 16);
                    // the same operations as the validity test above
                    const float pc_rot = pj * cos_t - pi * sin_t;
                    const float pr_rot = pj * sin_t + pi * cos_t;
                    float rb = pr_rot + d / 2 - 0.5f;
                    float cb = pc_rot + d / 2 - 0.5f;
                    const int pr = ptiy + pi, pc = ptix + pj;
                    const float dx = DAT(img, cols, pr, pc + 1) - DAT(img, cols, pr, pc - 1);
                    const float dy = DAT(img, cols, pr - 1, pc) - DAT(img, cols, pr + 1, pc);
                    const float wgt = exp32f((pc_rot * pc_rot + pr_rot * pr_rot) * exp_scale, tab);
                    const float o = fast_atan2(dy, dx);
                    const float mag = sqrtf(dx * dx + dy * dy) * wgt;
                    float obin = (o - ori) * bins_per_rad;
                    int r0 = (int)floorf(rb), c0 = (int)floorf(cb), o0 = (int)floorf(obin);
                    rb -= r0; cb -= c0; obin -= o0;
                    if (o0 < 0) o0 += n;
                    if (o0 >= n) o0 -= n;
                    pidx[lane] = ((r0 + 1) * (d + 2) + c0 + 1) * (n + 2) + o0;
                    // slot order = bin offset order {0, 1, 10, 11, 60, 61, 70, 71}
                    const float v_r1 = mag * rb, v_r0 = mag - v_r1;
                    const float v_rc11 = v_r1 * cb, v_rc10 = v_r1 - v_rc11;
                    const float v_rc01 = v_r0 * cb, v_rc00 = v_r0 - v_rc01;
                    const float v_rco111 = v_rc11 * obin, v_rco110 = v_rc11 - v_rco111;
                    const float v_rco101 = v_rc10 * obin, v_rco100 = v_rc10 - v_rco101;
                    const float v_rco011 = v_rc01 * obin, v_rco010 = v_rc01 - v_rco011;
                    const float v_rco001 = v_rc00 * obin, v_rco000 = v_rc00 - v_rco001;
                    pval[0 * 72 + lane] = v_rco000; pval[1 * 72 + lane] = v_rco001;
                    pval[2 * 72 + lane] = v_rco010; pval[3 * 72 + lane] = v_rco011;
                    pval[4 * 72 + lane] = v_rco100; pval[5 * 72 + lane] = v_rco101;
                    pval[6 * 72 + lane] = v_rco110; pval[7 * 72 + lane] = v_rco111;
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                // walk the chunk's pixels in raster order.  Consecutive pixels with the same base
                // bin (common: the smoothed gradient changes slowly) form runs, cut into sub-runs
                // of at most four; a sub-run is one read-add-write of its eight bins by eight
                // lanes (lds_rmw_add4_lanes), sub-runs one after another, 8 per group: lane
                // 8*j + k serves sub-run g + j, bin offset k.  Each bin still receives its
                // additions one at a time in pixel order.
                {
                    const int my_idx = lane < take ? pidx[lane] : -1;
                    const int prv = __shfl_up(my_idx, 1, 64);
                    const uint64_t rs = __ballot(lane < take && (lane == 0 || my_idx != prv));   // run starts
                    const uint64_t upto = rs & (lane == 63 ? ~0ull : ((2ull << lane) - 1ull));
                    const int last = 63 - __clzll((long long)upto);                             // this run's start
                    const uint64_t ss = __ballot(lane < take && ((lane - last) & 3) == 0);       // sub-run starts
                    if ((ss >> lane) & 1ull) slist[__popcll(ss & ((1ull << lane) - 1ull))] = lane;
                    const int ns = __popcll(ss);
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    for (int g = 0; g < ns; g += 8) {
                        const int rr = g + (lane >> 3), k = lane & 7;
                        const bool act = rr < ns;
                        const int koff = (0x4746'3D3C'0B0A'0100ull >> (8 * k)) & 0xFF;   // {0,1,10,11,60,61,70,71}
                        // every read unconditional and in bounds (sub-run index clamped, s0 + 3 <= 66
                        // < the 72-float row), then selects: no exec-mask dance per conditional
                        // read.  Inactive lanes' values are never used (the walk masks them out);
                        // an active lane's missing pixels are exact +0 by the selects.
                        const int rrc = act ? rr : 0;
                        const int s0 = slist[rrc];
                        const int s1 = slist[min(rrc + 1, 63)];
                        const int e0 = rrc + 1 < ns ? s1 : take;
                        const int m = e0 - s0;                                           // 1..4 if active
                        const int addr = pidx[s0] + koff;
                        const float* pv = pval + k * 72 + s0;
                        const float p0 = pv[0], p1 = pv[1], p2 = pv[2], p3 = pv[3];
                        const float v0 = p0;
                        const float v1 = m > 1 ? p1 : 0.f;
                        const float v2 = m > 2 ? p2 : 0.f;
                        const float v3 = m > 3 ? p3 : 0.f;
                        const uint64_t am = __ballot(act);
                        lds_rmw_add4_walk8(hist + addr, v0, v1, v2, v3, am);
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                head = (head + take) & 127;
                pend -= take;
            }
        }
        // circular orientation wrap + copy (independent per output)
        for (int t = lane; t < d * d * n; t += 64) {
            const int cell = t / n, k = t - cell * n;
            const int i = cell / d, j = cell - i * d;
            const int idx = ((i + 1) * (d + 2) + (j + 1)) * (n + 2);
            float v = hist[idx + k];
            if (k < 2) v += hist[idx + n + k];
            dsl[t] = v;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // the two norms: every square is formed per lane (the same rounded products), only the
        // 128 additions stay sequential on lane 0, in the serial order
        const int len = d * d * n;
        float* sq = pval_s[w] + 128;
        for (int t = lane; t < len; t += 64) sq[t] = dsl[t] * dsl[t];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane == 0) {
            float nrm2 = 0;
            for (int k = 0; k < len; ++k) nrm2 += sq[k];
            red_s[w][0] = sqrtf(nrm2) * SIFT_DESCR_MAG_THR;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const float thr = red_s[w][0];
        for (int t = lane; t < len; t += 64) {
            const float v = dsl[t] < thr ? dsl[t] : thr;
            sq[t] = v * v;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane == 0) {
            float nrm2 = 0;
            for (int k = 0; k < len; ++k) nrm2 += sq[k];
            red_s[w][1] = nrm2;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const float s2 = sqrtf(red_s[w][1]);
        const float nscale = SIFT_INT_DESCR_FCTR / (s2 > FLT_EPSILON ? s2 : FLT_EPSILON);
        float* dst = im.desc + 128 * (int64_t)q;
        for (int t = lane; t < len; t += 64) {
            const float v = dsl[t] < thr ? dsl[t] : thr;
            const int iv = __float2int_rn(v * nscale);
            dst[t] = (float)(iv < 0 ? 0 : (iv > 255 ? 255 : iv));
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// ratio test + gathering (:218-245), ordered by query index
__global__ void __launch_bounds__(256) k_ratio(const float* kp0, const float* kp1, int kps, const int32_t* idx2,
                                              const float* dist2, const int32_t* nq_p, int qs, double ratio,
                                              float* pts0, float* pts1, int32_t* counts, int cap)
{
    __shared__ int lds[16];
    const int b = blockIdx.x, tid = threadIdx.x;
    const int nq = nq_p[b];
    const float* k0 = kp0 + (int64_t)b * kps * 6;
    const float* k1 = kp1 + (int64_t)b * kps * 6;
    const int32_t* ix = idx2 + (int64_t)b * qs * 2;
    const float* dd = dist2 + (int64_t)b * qs * 2;
    float* a0 = pts0 + (int64_t)b * cap * 2;
    float* a1 = pts1 + (int64_t)b * cap * 2;
    int out = 0;
    for (int base = 0; base < nq; base += blockDim.x) {
        const int i = base + tid;
        bool keep = false;
        if (i < nq && ix[2 * i] >= 0 && ix[2 * i + 1] >= 0)
            keep = (double)dd[2 * i] < ratio * (double)dd[2 * i + 1];
        int tot;
        const int pos = out + block_scan_flag(keep, lds, &tot);
        if (keep && pos < cap) {
            a0[2 * pos] = k0[6 * i]; a0[2 * pos + 1] = k0[6 * i + 1];
            const int j = ix[2 * i];
            a1[2 * pos] = k1[6 * j]; a1[2 * pos + 1] = k1[6 * j + 1];
        }
        out += tot;
    }
    if (tid == 0) counts[b] = out < cap ? out : cap;
}

}  // namespace

// ======================================================================= host side
#define VO_STREAM(s) ((hipStream_t)(s))
static inline int hip_rc() { return hipGetLastError() == hipSuccess ? VO_OK : VO_EHIP; }

extern "C" int vo_sift_plan(vo_sift_buf* sb, int W, int H)
{
    if (!sb || W < 1 || H < 1) return VO_EARG;
    sb->W = W;
    sb->H = H;
    sb->nfeatures = 0;
    const int bw = 2 * W, bh = 2 * H;
    const int mn = bw < bh ? bw : bh;
    int n_oct = (int)lrint(log((double)mn) / log(2.) - 2) + 1;
    if (n_oct > VO_SIFT_MAX_OCT) n_oct = VO_SIFT_MAX_OCT;
    if (n_oct < 1) n_oct = 1;
    sb->n_oct = n_oct;
    int64_t go = 0, doff = 0;
    int w = bw, h = bh;
    for (int o = 0; o < n_oct; ++o) {
        if (o > 0) { w = w / 2; h = h / 2; }
        sb->oct_w[o] = w;
        sb->oct_h[o] = h;
        for (int i = 0; i < N_LAYERS + 3; ++i) { sb->gauss_off[o * 6 + i] = go; go += (int64_t)w * h; }
        for (int i = 0; i < N_LAYERS + 2; ++i) { sb->dog_off[o * 5 + i] = doff; doff += (int64_t)w * h; }
    }
    sb->gauss_floats = go;
    sb->dog_floats = doff;
    sb->tmp_floats = (int64_t)bw * bh;
    return VO_OK;
}

static int gauss_ksize(double sigma) { return ((int)lrint(sigma * 4 * 2 + 1)) | 1; }

static void gauss_kernel(int n, double sigma, float* k)
{
    double s2 = -0.5 / (sigma * sigma), sum = 0;
    for (int i = 0; i < n; ++i) {
        double x = i - (n - 1) * 0.5;
        k[i] = (float)exp(s2 * x * x);
        sum += k[i];
    }
    sum = 1. / sum;
    for (int i = 0; i < n; ++i) k[i] = (float)(k[i] * sum);
}

// blocks per image of the wave-per-keypoint kernels (they loop over their items)
#define SIFT_WAVE_BLOCKS 512

extern "C" int vo_sift_batch(const vo_sift_buf* sb, int B, const uint8_t* imgs, int64_t img_stride, int W, int H,
                             vo_stream_t stream)
{
    if (!sb || !imgs || B < 1 || B > 65535 || sb->W != W || sb->H != H || !sb->gauss || !sb->dog || !sb->tmp ||
        !sb->consts || img_stride < (int64_t)W * H || sb->kp_cap < 1 || sb->kp_cap > SORT_N || sb->nfeatures < 0 ||
        (sb->nfeatures > 0 && (int64_t)sb->cand_cap * 4 < 4 * (int64_t)sb->kp_cap + 2))
        return VO_EARG;
    hipStream_t st = VO_STREAM(stream);
    // host-side constants with the C library's exp/pow (as the oracle): kernel 0 = base blur,
    // kernels 1..5 = layer increments, then the exp32f table.  They depend on nothing but the
    // SIFT defaults, so they are built once into pinned host memory (thread-safe static init)
    // and uploaded stream-ordered: work still queued on `st` may be touching sb->consts.
    struct SiftConsts {
        float* host = nullptr;
        int ks[N_LAYERS + 3];
        bool ok = false;
        SiftConsts()
        {
            if (hipHostMalloc((void**)&host, sizeof(float) * (EXPTAB_OFF + 64)) != hipSuccess) return;
            memset(host, 0, sizeof(float) * (EXPTAB_OFF + 64));
            const double sigma = 1.6;
            const float sig_diff = sqrtf(fmaxf((float)(sigma * sigma) - 0.5f * 0.5f * 4, 0.01f));
            ks[0] = gauss_ksize(sig_diff);
            double sig[N_LAYERS + 3];
            sig[0] = sigma;
            const double k = pow(2., 1. / N_LAYERS);
            for (int i = 1; i < N_LAYERS + 3; ++i) {
                double sig_prev = pow(k, (double)(i - 1)) * sigma;
                double sig_total = sig_prev * k;
                sig[i] = sqrt(sig_total * sig_total - sig_prev * sig_prev);
            }
            for (int i = 1; i < N_LAYERS + 3; ++i) ks[i] = gauss_ksize(sig[i]);
            for (int i = 0; i < N_LAYERS + 3; ++i)
                if (ks[i] > KTAPS) return;
            gauss_kernel(ks[0], sig_diff, host);
            for (int i = 1; i < N_LAYERS + 3; ++i) gauss_kernel(ks[i], sig[i], host + i * KTAPS);
            for (int i = 0; i < 64; ++i) host[EXPTAB_OFF + i] = (float)(pow(2.0, i / 64.0) * EXPPOLY_32F_A0);
            ok = true;
        }
    };
    static const SiftConsts SC;
    if (!SC.ok) return VO_EHIP;
    const int* ks = SC.ks;
    if (hipMemcpyAsync(sb->consts, SC.host, sizeof(float) * (EXPTAB_OFF + 64), hipMemcpyHostToDevice, st) != hipSuccess)
        return VO_EHIP;
    if (hipMemsetAsync(sb->counters, 0, 8 * sizeof(int32_t) * (size_t)B, st) != hipSuccess) return VO_EHIP;
    const unsigned nb = (unsigned)B;
    const int64_t gs = sb->gauss_floats, ds = sb->dog_floats;
    // base: 2x upsample (into the blur scratch) + blur to sigma
    hipLaunchKernelGGL(k_upsample, dim3((2 * W + 255) / 256, (2 * H + UP_ROWS - 1) / UP_ROWS, nb), dim3(256), 0, st, imgs,
                       img_stride, W, H,
                       sb->tmp, sb->tmp_floats);
    auto blur = [&](const float* src, int64_t src_stride, float* dst, float* dog, int w, int h, int layer) {
        dim3 g((w + BT_W - 1) / BT_W, (h + BT_H - 1) / BT_H, nb);
        const float* kern = sb->consts + layer * KTAPS;
        // packed compile-time-size form for the SIFT kernel sizes (VO_SIFT_BLUR_GENERIC=1: the
        // runtime-size kernel; both identical)
        static const bool generic = [] { const char* e = getenv("VO_SIFT_BLUR_GENERIC"); return e && atoi(e) == 1; }();
        switch (generic ? 0 : ks[layer]) {
        case 11: hipLaunchKernelGGL(k_blur_tile_n<11>, g, dim3(256), 0, st, src, src_stride, dst, gs, dog, ds, w, h, kern); return;
        case 13: hipLaunchKernelGGL(k_blur_tile_n<13>, g, dim3(256), 0, st, src, src_stride, dst, gs, dog, ds, w, h, kern); return;
        case 17: hipLaunchKernelGGL(k_blur_tile_n<17>, g, dim3(256), 0, st, src, src_stride, dst, gs, dog, ds, w, h, kern); return;
        case 21: hipLaunchKernelGGL(k_blur_tile_n<21>, g, dim3(256), 0, st, src, src_stride, dst, gs, dog, ds, w, h, kern); return;
        case 27: hipLaunchKernelGGL(k_blur_tile_n<27>, g, dim3(256), 0, st, src, src_stride, dst, gs, dog, ds, w, h, kern); return;
        default: break;
        }
        const int rr = ks[layer] >> 1;
        const size_t lds = sizeof(float) * (size_t)(BT_H + 2 * rr) * (BT_W + 2 * rr + 1 + BT_W);
        hipLaunchKernelGGL(k_blur_tile, g, dim3(256), lds, st, src, src_stride, dst, gs, dog, ds, w, h, kern, ks[layer]);
    };
    blur(sb->tmp, sb->tmp_floats, sb->gauss + sb->gauss_off[0], nullptr, 2 * W, 2 * H, 0);
    for (int o = 0; o < sb->n_oct; ++o) {
        const int w = sb->oct_w[o], h = sb->oct_h[o];
        if (w < 1 || h < 1) continue;
        if (o > 0) {
            const float* src = sb->gauss + sb->gauss_off[(o - 1) * 6 + N_LAYERS];
            hipLaunchKernelGGL(k_nn_down, dim3((w + 127) / 128, h, nb), dim3(128), 0, st, src, sb->oct_w[o - 1],
                               sb->oct_h[o - 1], sb->gauss + sb->gauss_off[o * 6], w, h, gs);
        }
        // G_i = blur(G_{i-1}); the same pass writes D_{i-1} = G_i - G_{i-1}.  The top layer
        // G_{N_LAYERS+2} is only ever read through its DoG (keypoints live on layers 1..N_LAYERS,
        // the next octave starts from G_{N_LAYERS}), so that pass writes the DoG alone
        for (int i = 1; i < N_LAYERS + 3; ++i)
            blur(sb->gauss + sb->gauss_off[o * 6 + i - 1], gs,
                 i < N_LAYERS + 2 ? sb->gauss + sb->gauss_off[o * 6 + i] : nullptr,
                 sb->dog + sb->dog_off[o * 5 + i - 1], w, h, i);
    }
    for (int o = 0; o < sb->n_oct; ++o) {
        const int w = sb->oct_w[o], h = sb->oct_h[o];
        if (w <= 2 * SIFT_IMG_BORDER || h <= 2 * SIFT_IMG_BORDER) continue;
        // tiled, all layers of the octave per launch
        const dim3 g((w - 2 * SIFT_IMG_BORDER + EX_W - 1) / EX_W, (h - 2 * SIFT_IMG_BORDER + EX_H - 1) / EX_H, nb);
        hipLaunchKernelGGL(k_extrema_t, g, dim3(256), 0, st, *sb, o);
    }
    hipLaunchKernelGGL(k_sift_refine, dim3((sb->cand_cap + 127) / 128, 1, nb), dim3(128), 0, st, *sb);
    hipLaunchKernelGGL(k_sift_ori, dim3(SIFT_WAVE_BLOCKS, 1, nb), dim3(256), 0, st, *sb);
    hipLaunchKernelGGL(k_sift_sort_dedupe, dim3(1, 1, nb), dim3(1024), 0, st, *sb);
    if (sb->nfeatures > 0)
        hipLaunchKernelGGL(k_sift_retain_best, dim3(1, 1, nb), dim3(RB_T), 0, st, *sb);
    hipLaunchKernelGGL(k_sift_desc_w, dim3(SIFT_WAVE_BLOCKS, 1, nb), dim3(256), 0, st, *sb);
    return hip_rc();
}

// Test hook: k_sift_retain_best on caller-given keypoint rows, so its partition
// rounds can be pinned against libstdc++ on tie-heavy and adversarial response arrays (the
// SIFT scenes rarely reach them).  counters[2] must hold n on entry and holds the kept count
// on return; kp_out [n][6] (response in column 4) is reordered in place; scratch >= 4 n + 2
// ints, tmp >= 6 n floats.
extern "C" int vo_sift_retain_best_rows(float* kp_out, int32_t n, int32_t nfeatures, int32_t* counters,
                                        int32_t* scratch, float* tmp, vo_stream_t stream)
{
    if (!kp_out || !counters || !scratch || !tmp || n < 0 || n > 32768) return VO_EARG;
    vo_sift_buf sb;
    memset(&sb, 0, sizeof sb);
    sb.counters = counters;
    sb.cand = scratch;
    sb.cand_cap = n + 1;                        // 4 cand_cap ints >= 4 n + 2 (rec, LP, RP)
    sb.kp = tmp;
    sb.kp_out = kp_out;
    sb.kp_cap = n;
    sb.nfeatures = nfeatures;
    hipLaunchKernelGGL(k_sift_retain_best, dim3(1, 1, 1), dim3(RB_T), 0, (hipStream_t)stream, sb);
    return hip_rc();
}

extern "C" int vo_sift(const vo_sift_buf* sb, const uint8_t* img, int W, int H, vo_stream_t stream)
{
    return vo_sift_batch(sb, 1, img, (int64_t)W * H, W, H, stream);
}

extern "C" int vo_ratio_matches(int B, const float* kp0, const float* kp1, int32_t kp_stride, const int32_t* idx2,
                                const float* dist2, const int32_t* nq, int32_t q_stride, double ratio, float* pts0,
                                float* pts1, int32_t* counts, int32_t cap, vo_stream_t stream)
{
    if (B < 1 || !kp0 || !kp1 || !idx2 || !dist2 || !nq || !pts0 || !pts1 || !counts) return VO_EARG;
    hipLaunchKernelGGL(k_ratio, dim3(B), dim3(256), 0, VO_STREAM(stream), kp0, kp1, kp_stride, idx2, dist2, nq, q_stride,
                       ratio, pts0, pts1, counts, cap);
    return hip_rc();
}
