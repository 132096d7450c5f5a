/*
 * vo_oracle_img.c -- CPU ORACLE (test infrastructure only; see vo_oracle.h).
 *
 * Restates, for the reference call sites:
 *   VisualOdometryPipeLine.py:256  cv2.goodFeaturesToTrack   
 *   VisualOdometryPipeLine.py:281,287 cv2.calcOpticalFlowPyrLK
 *
 * Deliberate, documented deviations from OpenCV 4.6 (identical in the HIP path):
 *   - GFTT: Sobel, covariance and box sums are computed exactly in integers and
 *     lambda_min in fp64 from those integers, then rounded to float (OpenCV forms
 *     Sobel*scale in fp32 and box-sums in fp64).  The ordering rule (value desc,
 *     then larger address first) and the greedy grid test are OpenCV's.
 *   - LK: window sums A11/A12/A22/b1/b2 are accumulated exactly in int64 and
 *     converted to float once (OpenCV accumulates in fp32, lane-order dependent).
 *
 * vo_o_set_fp32_mode() switches on restatements of OpenCV's fp32 forms instead (never used
 * by the parity tests; tools/opencv_fp32_sensitivity.py measures how often they change a
 * result): bit 0 -- cornerMinEigenVal as Sobel * scale in float (scale on the smoothing
 * taps), float covariance products, double box sums rounded to float, lambda in float
 * (corner.cpp); bit 1 -- LK sums accumulated in float in raster order (lkpyramid.cpp's
 * scalar loop).  OpenCV's SIMD builds may fuse and reorder these; unpinned either way.
 */
#include "vo_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ RNG */
uint32_t vo_o_rng_next(uint64_t* state)
{
    /* cv::RNG::next(): state = (uint64)(unsigned)state * 4164903690 + (state >> 32) */
    uint64_t s = *state;
    s = (uint64_t)(uint32_t)s * 4164903690ULL + (s >> 32);
    *state = s;
    return (uint32_t)s;
}

static inline int refl101(int p, int len)
{
    if (len == 1) return 0;
    while (p < 0 || p >= len) {
        if (p < 0) p = -p;
        else p = 2 * len - p - 2;
    }
    return p;
}

static int g_fp32_mode = 0;
void vo_o_set_fp32_mode(int mode) { g_fp32_mode = mode; }

/* OpenCV-style fp32 cornerMinEigenVal (bit 0 of the fp32 mode), blockSize x blockSize, ksize 3 */
static int eigmap_fp32(const uint8_t* img, int w, int h, int bs, float* eig)
{
    size_t npx = (size_t)w * h;
    float* cov = (float*)malloc(npx * 3 * sizeof(float));
    if (!cov) return VO_O_EFAIL;
    const double scale = 1.0 / ((double)(1 << 2) * bs * 255.0);
    const float k0 = (float)(1.0 * scale), k1 = (float)(2.0 * scale);   /* smoothing taps * scale */
    for (int y = 0; y < h; ++y) {
        int ym = refl101(y - 1, h), yp = refl101(y + 1, h);
        for (int x = 0; x < w; ++x) {
            int xm = refl101(x - 1, w), xp = refl101(x + 1, w);
            const uint8_t* r0 = img + (size_t)ym * w;
            const uint8_t* r1 = img + (size_t)y * w;
            const uint8_t* r2 = img + (size_t)yp * w;
            /* dx: row difference, then the (1 2 1)*scale column pass; dy: row smoothing
               (1 2 1) then the column difference, scaled by the smoothing taps */
            float d0 = (float)(r0[xp] - r0[xm]), d1 = (float)(r1[xp] - r1[xm]), d2 = (float)(r2[xp] - r2[xm]);
            float dxf = (d0 + d2) * k0 + d1 * k1;
            float s0 = (float)r0[xm] * k0 + (float)r0[x] * k1 + (float)r0[xp] * k0;
            float s2 = (float)r2[xm] * k0 + (float)r2[x] * k1 + (float)r2[xp] * k0;
            float dyf = s2 - s0;
            cov[3 * ((size_t)y * w + x)] = dxf * dxf;
            cov[3 * ((size_t)y * w + x) + 1] = dxf * dyf;
            cov[3 * ((size_t)y * w + x) + 2] = dyf * dyf;
        }
    }
    int a0 = bs / 2;
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            double sa = 0, sb = 0, sc = 0;
            for (int i = 0; i < bs; ++i) {
                int yy = refl101(y - a0 + i, h);
                for (int j = 0; j < bs; ++j) {
                    int xx = refl101(x - a0 + j, w);
                    const float* c = cov + 3 * ((size_t)yy * w + xx);
                    sa += c[0]; sb += c[1]; sc += c[2];
                }
            }
            float a = (float)sa * 0.5f, b = (float)sb, c = (float)sc * 0.5f;
            eig[(size_t)y * w + x] = (float)((a + c) - sqrtf((a - c) * (a - c) + b * b));
        }
    free(cov);
    return VO_O_OK;
}

/* ------------------------------------------------------------------ GFTT */
int vo_o_eigmap(const uint8_t* img, int w, int h, int bs, int use_harris,
                double harris_k, float* eig)
{
    if (!img || w < 1 || h < 1 || bs < 1 || !eig) return VO_O_EARG;
    if ((g_fp32_mode & 1) && !use_harris) return eigmap_fp32(img, w, h, bs, eig);
    size_t npx = (size_t)w * h;
    int32_t* dx = (int32_t*)malloc(npx * sizeof(int32_t));
    int32_t* dy = (int32_t*)malloc(npx * sizeof(int32_t));
    if (!dx || !dy) { free(dx); free(dy); return VO_O_EFAIL; }
    /* Sobel 3x3, BORDER_REFLECT_101 (corner.cpp cornerEigenValsVecs) */
    for (int y = 0; y < h; ++y) {
        int ym = refl101(y - 1, h), yp = refl101(y + 1, h);
        for (int x = 0; x < w; ++x) {
            int xm = refl101(x - 1, w), xp = refl101(x + 1, w);
            const uint8_t* r0 = img + (size_t)ym * w;
            const uint8_t* r1 = img + (size_t)y * w;
            const uint8_t* r2 = img + (size_t)yp * w;
            int gx = (r0[xp] - r0[xm]) + 2 * (r1[xp] - r1[xm]) + (r2[xp] - r2[xm]);
            int gy = (r2[xm] - r0[xm]) + 2 * (r2[x] - r0[x]) + (r2[xp] - r0[xp]);
            dx[(size_t)y * w + x] = gx;
            dy[(size_t)y * w + x] = gy;
        }
    }
    /* unnormalised block box sum of (dx^2, dxdy, dy^2), anchor at block centre,
       BORDER_REFLECT_101 on the covariance image */
    const double s = 1.0 / ((double)(1 << 2) * bs * 255.0);
    const double lam_scale = s * s * 0.5;
    const double har_scale = s * s * s * s;
    int a0 = bs / 2;
    for (int y = 0; y < h; ++y) {
        for (int x = 0; x < w; ++x) {
            int64_t sxx = 0, sxy = 0, syy = 0;
            for (int i = 0; i < bs; ++i) {
                int yy = refl101(y - a0 + i, h);
                for (int j = 0; j < bs; ++j) {
                    int xx = refl101(x - a0 + j, w);
                    int64_t gx = dx[(size_t)yy * w + xx], gy = dy[(size_t)yy * w + xx];
                    sxx += gx * gx;
                    sxy += gx * gy;
                    syy += gy * gy;
                }
            }
            float v;
            if (!use_harris) {
                int64_t T = sxx + syy;
                int64_t dd = sxx - syy;
                int64_t D = dd * dd + 4 * sxy * sxy;
                double lam = ((double)T - sqrt((double)D)) * lam_scale;
                v = (float)lam;
            } else {
                int64_t det = sxx * syy - sxy * sxy;
                int64_t T = sxx + syy;
                double r = ((double)det - harris_k * (double)(T * T)) * har_scale;
                v = (float)r;
            }
            eig[(size_t)y * w + x] = v;
        }
    }
    free(dx);
    free(dy);
    return VO_O_OK;
}

typedef struct { float v; int32_t addr; } cand_t;

static int cand_cmp(const void* pa, const void* pb)
{
    /* greaterThanPtr: value desc, ties -> larger address first */
    const cand_t* a = (const cand_t*)pa;
    const cand_t* b = (const cand_t*)pb;
    if (a->v > b->v) return -1;
    if (a->v < b->v) return 1;
    return (a->addr > b->addr) ? -1 : (a->addr < b->addr) ? 1 : 0;
}

int vo_o_gftt(const uint8_t* img, int w, int h, int max_corners, double quality,
              double min_dist, int block_size, int use_harris, double harris_k,
              float* out_xy, int cap, int* out_n)
{
    if (!img || !out_n || w < 1 || h < 1) return VO_O_EARG;
    *out_n = 0;
    size_t npx = (size_t)w * h;
    float* eig = (float*)malloc(npx * sizeof(float));
    if (!eig) return VO_O_EFAIL;
    int rc = vo_o_eigmap(img, w, h, block_size, use_harris, harris_k, eig);
    if (rc) { free(eig); return rc; }
    double maxv = -DBL_MAX;
    for (size_t i = 0; i < npx; ++i) if (eig[i] > maxv) maxv = eig[i];
    float thr = (float)(maxv * quality);
    /* THRESH_TOZERO: keep v > thr */
    for (size_t i = 0; i < npx; ++i) if (!(eig[i] > thr)) eig[i] = 0.f;
    /* 3x3 dilate (border ignored) + collect v != 0 && v == dilated, x,y in [1, n-2] */
    cand_t* cands = (cand_t*)malloc(npx * sizeof(cand_t));
    if (!cands) { free(eig); return VO_O_EFAIL; }
    size_t nc = 0;
    for (int y = 1; y < h - 1; ++y) {
        for (int x = 1; x < w - 1; ++x) {
            float v = eig[(size_t)y * w + x];
            if (v == 0.f) continue;
            float m = v;
            for (int dy = -1; dy <= 1; ++dy)
                for (int dx = -1; dx <= 1; ++dx) {
                    float u = eig[(size_t)(y + dy) * w + (x + dx)];
                    if (u > m) m = u;
                }
            if (v == m) {
                cands[nc].v = v;
                cands[nc].addr = y * w + x;
                ++nc;
            }
        }
    }
    free(eig);
    if (nc == 0) { free(cands); return VO_O_OK; }
    qsort(cands, nc, sizeof(cand_t), cand_cmp);

    int ncorners = 0;
    if (min_dist >= 1) {
        int cell = (int)lrint(min_dist);               /* cvRound */
        int gw = (w + cell - 1) / cell, gh = (h + cell - 1) / cell;
        /* per cell: dynamic list of accepted points */
        int* head = (int*)malloc(sizeof(int) * (size_t)gw * gh);
        int* next = (int*)malloc(sizeof(int) * nc);
        float* ax = (float*)malloc(sizeof(float) * nc);
        float* ay = (float*)malloc(sizeof(float) * nc);
        for (int i = 0; i < gw * gh; ++i) head[i] = -1;
        double md2 = min_dist * min_dist;
        int nacc = 0;
        for (size_t i = 0; i < nc; ++i) {
            int y = cands[i].addr / w, x = cands[i].addr - (cands[i].addr / w) * w;
            int xc = x / cell, yc = y / cell;
            int x1 = xc - 1 < 0 ? 0 : xc - 1, y1 = yc - 1 < 0 ? 0 : yc - 1;
            int x2 = xc + 1 > gw - 1 ? gw - 1 : xc + 1, y2 = yc + 1 > gh - 1 ? gh - 1 : yc + 1;
            int good = 1;
            for (int yy = y1; yy <= y2 && good; ++yy)
                for (int xx = x1; xx <= x2 && good; ++xx)
                    for (int k = head[yy * gw + xx]; k >= 0; k = next[k]) {
                        float ddx = (float)x - ax[k];
                        float ddy = (float)y - ay[k];
                        if ((double)(ddx * ddx + ddy * ddy) < md2) { good = 0; break; }
                    }
            if (!good) continue;
            ax[nacc] = (float)x;
            ay[nacc] = (float)y;
            next[nacc] = head[yc * gw + xc];
            head[yc * gw + xc] = nacc;
            ++nacc;
            if (ncorners < cap && out_xy) {
                out_xy[2 * ncorners] = (float)x;
                out_xy[2 * ncorners + 1] = (float)y;
            }
            ++ncorners;
            if (max_corners > 0 && ncorners == max_corners) break;
        }
        free(head); free(next); free(ax); free(ay);
    } else {
        for (size_t i = 0; i < nc; ++i) {
            int y = cands[i].addr / w, x = cands[i].addr % w;
            if (ncorners < cap && out_xy) {
                out_xy[2 * ncorners] = (float)x;
                out_xy[2 * ncorners + 1] = (float)y;
            }
            ++ncorners;
            if (max_corners > 0 && ncorners == max_corners) break;
        }
    }
    free(cands);
    *out_n = ncorners;
    return ncorners > cap ? VO_O_ECAP : VO_O_OK;
}

/* ------------------------------------------------------------------ pyramid */
int vo_o_pyrdown(const uint8_t* src, int w, int h, uint8_t* dst)
{
    if (!src || !dst || w < 1 || h < 1) return VO_O_EARG;
    static const int k5[5] = {1, 4, 6, 4, 1};
    int dw = (w + 1) / 2, dh = (h + 1) / 2;
    for (int y = 0; y < dh; ++y) {
        for (int x = 0; x < dw; ++x) {
            int acc = 0;
            for (int i = 0; i < 5; ++i) {
                const uint8_t* row = src + (size_t)refl101(2 * y - 2 + i, h) * w;
                int racc = 0;
                for (int j = 0; j < 5; ++j) racc += k5[j] * row[refl101(2 * x - 2 + j, w)];
                acc += k5[i] * racc;
            }
            dst[(size_t)y * dw + x] = (uint8_t)((acc + 128) >> 8);
        }
    }
    return VO_O_OK;
}

int vo_o_scharr(const uint8_t* src, int w, int h, int16_t* dst)
{
    if (!src || !dst || w < 1 || h < 1) return VO_O_EARG;
    for (int y = 0; y < h; ++y) {
        int y0 = y > 0 ? y - 1 : (h > 1 ? 1 : 0);
        int y2 = y < h - 1 ? y + 1 : (h > 1 ? h - 2 : 0);
        const uint8_t* s0 = src + (size_t)y0 * w;
        const uint8_t* s1 = src + (size_t)y * w;
        const uint8_t* s2 = src + (size_t)y2 * w;
        for (int x = 0; x < w; ++x) {
            int xl = x > 0 ? x - 1 : (w > 1 ? 1 : 0);
            int xr = x < w - 1 ? x + 1 : (w > 1 ? w - 2 : 0);
            /* vertical (3,10,3) smoothing for Ix, vertical difference for Iy */
            int t0l = (s0[xl] + s2[xl]) * 3 + s1[xl] * 10;
            int t0r = (s0[xr] + s2[xr]) * 3 + s1[xr] * 10;
            int t1l = s2[xl] - s0[xl], t1c = s2[x] - s0[x], t1r = s2[xr] - s0[xr];
            dst[((size_t)y * w + x) * 2] = (int16_t)(t0r - t0l);
            dst[((size_t)y * w + x) * 2 + 1] = (int16_t)((t1r + t1l) * 3 + t1c * 10);
        }
    }
    return VO_O_OK;
}

int vo_o_pyr_maxlevel(int w, int h, int win_w, int win_h, int max_level)
{
    /* buildOpticalFlowPyramid: stop when the next level is <= winSize */
    int lvl = 0;
    int sw = w, sh = h;
    for (lvl = 0; lvl <= max_level; ++lvl) {
        sw = (sw + 1) / 2;
        sh = (sh + 1) / 2;
        if (sw <= win_w || sh <= win_h) return lvl;
    }
    return max_level;
}

typedef struct {
    int w, h, bx, by, pw;   /* interior size, border, padded pitch */
    uint8_t* img;           /* padded (h+2by) x pw, reflect-101 border */
    int16_t* der;           /* padded, 2 int16 per px, zero border */
} lk_level_t;

static void pad_reflect(const uint8_t* src, int w, int h, int bx, int by, uint8_t* dst)
{
    int pw = w + 2 * bx;
    for (int y = -by; y < h + by; ++y) {
        const uint8_t* row = src + (size_t)refl101(y, h) * w;
        uint8_t* d = dst + (size_t)(y + by) * pw;
        for (int x = -bx; x < w + bx; ++x) d[x + bx] = row[refl101(x, w)];
    }
}

static int build_levels(const uint8_t* img, int w, int h, int bx, int by, int L,
                        lk_level_t* lv, int with_deriv)
{
    const uint8_t* cur = img;
    uint8_t* tmp = NULL;
    int cw = w, ch = h;
    for (int l = 0; l <= L; ++l) {
        uint8_t* interior;
        if (l == 0) {
            interior = (uint8_t*)malloc((size_t)cw * ch);
            memcpy(interior, img, (size_t)cw * ch);
        } else {
            int nw = (cw + 1) / 2, nh = (ch + 1) / 2;
            interior = (uint8_t*)malloc((size_t)nw * nh);
            vo_o_pyrdown(cur, cw, ch, interior);
            cw = nw; ch = nh;
        }
        lv[l].w = cw; lv[l].h = ch; lv[l].bx = bx; lv[l].by = by; lv[l].pw = cw + 2 * bx;
        lv[l].img = (uint8_t*)malloc((size_t)(ch + 2 * by) * lv[l].pw);
        pad_reflect(interior, cw, ch, bx, by, lv[l].img);
        lv[l].der = NULL;
        if (with_deriv) {
            int16_t* d = (int16_t*)malloc(sizeof(int16_t) * 2 * (size_t)cw * ch);
            vo_o_scharr(interior, cw, ch, d);
            lv[l].der = (int16_t*)calloc((size_t)(ch + 2 * by) * lv[l].pw * 2, sizeof(int16_t));
            for (int y = 0; y < ch; ++y)
                memcpy(lv[l].der + ((size_t)(y + by) * lv[l].pw + bx) * 2, d + (size_t)y * cw * 2,
                       sizeof(int16_t) * 2 * cw);
            free(d);
        }
        free(tmp);
        tmp = interior;
        cur = interior;
    }
    free(tmp);
    return 0;
}

static void free_levels(lk_level_t* lv, int L)
{
    for (int l = 0; l <= L; ++l) { free(lv[l].img); free(lv[l].der); }
}

#define DESCALE(x, n) (((x) + (1 << ((n)-1))) >> (n))

/* iteration histogram of the LK solver loop (diagnostics for kernel design; index =
 * iterations run at one level for one point, 0..100) */
int vo_o_lk_iter_hist[101];

int vo_o_lk(const uint8_t* prev, const uint8_t* next, int w, int h,
            const float* pts, int n, float* out_pts, uint8_t* status, float* err,
            int win_w, int win_h, int max_level, int crit_type, int max_count,
            double epsilon, double min_eig_thr)
{
    if (!prev || !next || (n > 0 && (!pts || !out_pts || !status))) return VO_O_EARG;
    if (win_w <= 2 || win_h <= 2 || max_level < 0) return VO_O_EARG;
    if (n == 0) return VO_O_OK;
    /* criteria normalisation (calcOpticalFlowPyrLK) */
    if (!(crit_type & 1)) max_count = 30;
    else max_count = max_count < 0 ? 0 : (max_count > 100 ? 100 : max_count);
    if (!(crit_type & 2)) epsilon = 0.01;
    else epsilon = epsilon < 0 ? 0 : (epsilon > 10 ? 10 : epsilon);
    epsilon *= epsilon;
    const float min_eig = (float)min_eig_thr;

    int L = vo_o_pyr_maxlevel(w, h, win_w, win_h, max_level);
    lk_level_t* P = (lk_level_t*)calloc((size_t)L + 1, sizeof(lk_level_t));
    lk_level_t* J = (lk_level_t*)calloc((size_t)L + 1, sizeof(lk_level_t));
    build_levels(prev, w, h, win_w, win_h, L, P, 1);
    build_levels(next, w, h, win_w, win_h, L, J, 0);

    const float hx = (win_w - 1) * 0.5f, hy = (win_h - 1) * 0.5f;
    const int W_BITS = 14;
    const float FLT_SCALE = 1.f / (1 << 20);
    int16_t* Iwin = (int16_t*)malloc(sizeof(int16_t) * (size_t)win_w * win_h);
    int16_t* dIwin = (int16_t*)malloc(sizeof(int16_t) * 2 * (size_t)win_w * win_h);

    for (int i = 0; i < n; ++i) status[i] = 1;
    for (int level = L; level >= 0; --level) {
        const lk_level_t* I = &P[level];
        const lk_level_t* Jl = &J[level];
        const int cols = I->w, rows = I->h;
        for (int pi = 0; pi < n; ++pi) {
            float sc = (float)(1. / (1 << level));
            float px = pts[2 * pi] * sc, py = pts[2 * pi + 1] * sc;
            float nx, ny;
            if (level == L) { nx = px; ny = py; }
            else { nx = out_pts[2 * pi] * 2.f; ny = out_pts[2 * pi + 1] * 2.f; }
            out_pts[2 * pi] = nx;
            out_pts[2 * pi + 1] = ny;

            px -= hx; py -= hy;
            int ipx = (int)floorf(px), ipy = (int)floorf(py);
            if (ipx < -win_w || ipx >= cols || ipy < -win_h || ipy >= rows) {
                if (level == 0) { status[pi] = 0; if (err) err[pi] = 0; }
                continue;
            }
            float a = px - ipx, b = py - ipy;
            int iw00 = (int)lrintf((1.f - a) * (1.f - b) * (1 << W_BITS));
            int iw01 = (int)lrintf(a * (1.f - b) * (1 << W_BITS));
            int iw10 = (int)lrintf((1.f - a) * b * (1 << W_BITS));
            int iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;
            int64_t iA11 = 0, iA12 = 0, iA22 = 0;
            float fA11 = 0.f, fA12 = 0.f, fA22 = 0.f;
            const int lk32 = g_fp32_mode & 2;
            for (int y = 0; y < win_h; ++y) {
                const uint8_t* src = I->img + (size_t)(y + ipy + I->by) * I->pw + (ipx + I->bx);
                const int16_t* dsrc = I->der + ((size_t)(y + ipy + I->by) * I->pw + (ipx + I->bx)) * 2;
                int dstep = I->pw * 2;
                for (int x = 0; x < win_w; ++x) {
                    int ival = DESCALE(src[x] * iw00 + src[x + 1] * iw01 + src[x + I->pw] * iw10 +
                                       src[x + I->pw + 1] * iw11, W_BITS - 5);
                    const int16_t* d = dsrc + 2 * x;
                    int ixval = DESCALE(d[0] * iw00 + d[2] * iw01 + d[dstep] * iw10 + d[dstep + 2] * iw11, W_BITS);
                    int iyval = DESCALE(d[1] * iw00 + d[3] * iw01 + d[dstep + 1] * iw10 + d[dstep + 3] * iw11, W_BITS);
                    Iwin[y * win_w + x] = (int16_t)ival;
                    dIwin[2 * (y * win_w + x)] = (int16_t)ixval;
                    dIwin[2 * (y * win_w + x) + 1] = (int16_t)iyval;
                    iA11 += (int64_t)ixval * ixval;
                    iA12 += (int64_t)ixval * iyval;
                    iA22 += (int64_t)iyval * iyval;
                    fA11 += (float)(ixval * ixval);
                    fA12 += (float)(ixval * iyval);
                    fA22 += (float)(iyval * iyval);
                }
            }
            float A11 = (lk32 ? fA11 : (float)iA11) * FLT_SCALE;
            float A12 = (lk32 ? fA12 : (float)iA12) * FLT_SCALE;
            float A22 = (lk32 ? fA22 : (float)iA22) * FLT_SCALE;
            float D = A11 * A22 - A12 * A12;
            float minEig = (A22 + A11 - sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) /
                           (float)(2 * win_w * win_h);
            if (minEig < min_eig || D < FLT_EPSILON) {
                if (level == 0) status[pi] = 0;
                continue;
            }
            D = 1.f / D;
            nx -= hx; ny -= hy;
            float pdx = 0.f, pdy = 0.f;
            int iters_run = 0;
            for (int j = 0; j < max_count; ++j) {
                iters_run = j + 1;
                int inx = (int)floorf(nx), iny = (int)floorf(ny);
                if (inx < -win_w || inx >= cols || iny < -win_h || iny >= rows) {
                    if (level == 0) status[pi] = 0;
                    break;
                }
                a = nx - inx; b = ny - iny;
                iw00 = (int)lrintf((1.f - a) * (1.f - b) * (1 << W_BITS));
                iw01 = (int)lrintf(a * (1.f - b) * (1 << W_BITS));
                iw10 = (int)lrintf((1.f - a) * b * (1 << W_BITS));
                iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;
                int64_t ib1 = 0, ib2 = 0;
                float fb1 = 0.f, fb2 = 0.f;
                for (int y = 0; y < win_h; ++y) {
                    const uint8_t* Jp = Jl->img + (size_t)(y + iny + Jl->by) * Jl->pw + (inx + Jl->bx);
                    for (int x = 0; x < win_w; ++x) {
                        int diff = DESCALE(Jp[x] * iw00 + Jp[x + 1] * iw01 + Jp[x + Jl->pw] * iw10 +
                                           Jp[x + Jl->pw + 1] * iw11, W_BITS - 5) - Iwin[y * win_w + x];
                        ib1 += (int64_t)diff * dIwin[2 * (y * win_w + x)];
                        ib2 += (int64_t)diff * dIwin[2 * (y * win_w + x) + 1];
                        fb1 += (float)(diff * dIwin[2 * (y * win_w + x)]);
                        fb2 += (float)(diff * dIwin[2 * (y * win_w + x) + 1]);
                    }
                }
                float b1 = (lk32 ? fb1 : (float)ib1) * FLT_SCALE;
                float b2 = (lk32 ? fb2 : (float)ib2) * FLT_SCALE;
                float ddx = (A12 * b2 - A22 * b1) * D;
                float ddy = (A12 * b1 - A11 * b2) * D;
                nx += ddx;
                ny += ddy;
                out_pts[2 * pi] = nx + hx;
                out_pts[2 * pi + 1] = ny + hy;
                if ((double)ddx * ddx + (double)ddy * ddy <= epsilon) break;
                if (j > 0 && fabsf(ddx + pdx) < 0.01f && fabsf(ddy + pdy) < 0.01f) {
                    out_pts[2 * pi] -= ddx * 0.5f;
                    out_pts[2 * pi + 1] -= ddy * 0.5f;
                    break;
                }
                pdx = ddx; pdy = ddy;
            }
            vo_o_lk_iter_hist[iters_run]++;
            if (status[pi] && err && level == 0) {
                float fx = out_pts[2 * pi] - hx, fy = out_pts[2 * pi + 1] - hy;
                int inx = (int)floorf(fx), iny = (int)floorf(fy);
                if (inx < -win_w || inx >= cols || iny < -win_h || iny >= rows) {
                    status[pi] = 0;
                    continue;
                }
                float aa = fx - inx, bb = fy - iny;
                iw00 = (int)lrintf((1.f - aa) * (1.f - bb) * (1 << W_BITS));
                iw01 = (int)lrintf(aa * (1.f - bb) * (1 << W_BITS));
                iw10 = (int)lrintf((1.f - aa) * bb * (1 << W_BITS));
                iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;
                float errval = 0.f;
                for (int y = 0; y < win_h; ++y) {
                    const uint8_t* Jp = Jl->img + (size_t)(y + iny + Jl->by) * Jl->pw + (inx + Jl->bx);
                    for (int x = 0; x < win_w; ++x) {
                        int diff = DESCALE(Jp[x] * iw00 + Jp[x + 1] * iw01 + Jp[x + Jl->pw] * iw10 +
                                           Jp[x + Jl->pw + 1] * iw11, W_BITS - 5) - Iwin[y * win_w + x];
                        errval += fabsf((float)diff);
                    }
                }
                err[pi] = errval / (float)(32 * win_w * win_h);
            }
        }
    }
    free(Iwin);
    free(dIwin);
    free_levels(P, L);
    free_levels(J, L);
    free(P);
    free(J);
    return VO_O_OK;
}
