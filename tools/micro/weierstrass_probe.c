#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <float.h>
#include <stdint.h>
static double g_co[200000][11]; static int g_nco = 0;
static void sp_hook(const double* c) { if (g_nco < 200000) { memcpy(g_co[g_nco], c, 11 * sizeof(double)); g_nco++; } }
#include "geom_hooked.c"

typedef struct { double re, im; } cx;
static int sweeps(const double* c_in, int* period, int* start)
{
    static cx hist[301][10];
    cplx co[11];
    for (int i = 0; i <= 10; ++i) { co[i].re = c_in[i]; co[i].im = 0; }
    int n = 10;
    for (; n > 1; --n) if (fabs(co[n].re) + fabs(co[n].im) > DBL_EPSILON) break;
    cplx p = {1, 0}, r = {1, 1}, roots[10];
    for (int i = 0; i < n; ++i) { roots[i] = p; p = c_mul(p, r); }
    memcpy(hist[0], roots, sizeof(cplx) * n);
    *period = 0; *start = -1;
    int iter;
    for (iter = 0; iter < 300; ++iter) {
        double maxDiff = 0;
        for (int i = 0; i < n; ++i) {
            p = roots[i];
            cplx num = co[n], denom = co[n];
            for (int j = 0; j < n; ++j) {
                num = c_add(c_mul(num, p), co[n - j - 1]);
                if (j != i) { cplx d = c_sub(p, roots[j]); if (!(d.re == 0 && d.im == 0)) denom = c_mul(denom, d); }
            }
            num = c_div(num, denom);
            roots[i] = c_sub(p, num);
            double a = sqrt(num.re * num.re + num.im * num.im);
            if (a > maxDiff) maxDiff = a;
        }
        memcpy(hist[iter + 1], roots, sizeof(cplx) * n);
        if (*start < 0)
            for (int k = iter; k >= 0 && k >= iter - 150; --k)
                if (!memcmp(hist[k], roots, sizeof(cplx) * n)) { *start = k; *period = iter + 1 - k; break; }
        if (maxDiff <= 0) break;
    }
    return iter + 1;
}

static double urand(uint64_t* s) { *s = *s * 6364136223846793005ULL + 1442695040888963407ULL; return (double)(*s >> 11) / 9007199254740992.0; }

int main(int argc, char** argv)
{
    uint64_t s = 12345;
    const double K[9] = {718.856, 0, 607.1928, 0, 718.856, 185.2157, 0, 0, 1};
    int nprob = argc > 1 ? atoi(argv[1]) : 20;
    double outl = argc > 2 ? atof(argv[2]) : 0.3;
    if (argc > 3) {
        for (int f = 0; f < nprob; ++f) {
            char nm[64]; sprintf(nm, "/tmp/wk/m_%d.bin", f);
            FILE* fp = fopen(nm, "rb"); float buf[4 * 8000]; int n = fread(buf, 16, 8000, fp); fclose(fp);
            float* p0 = malloc(8 * n); float* p1 = malloc(8 * n); uint8_t* mask = malloc(n);
            for (int i = 0; i < n; ++i) { p0[2*i] = buf[4*i]; p0[2*i+1] = buf[4*i+1]; p1[2*i] = buf[4*i+2]; p1[2*i+1] = buf[4*i+3]; }
            double E[9]; int nm_, before = g_nco;
            vo_o_find_essential(p0, p1, n, K, 0.999, 1.0, 1000, E, mask, &nm_);
            int inl = 0; for (int i = 0; i < n; ++i) inl += mask[i];
            fprintf(stderr, "file %d: n %d inliers %d hypotheses %d\n", f, n, inl, g_nco - before);
        }
        nprob = 0;
    }
    for (int pb = 0; pb < nprob; ++pb) {
        int n = 1500;
        float* p0 = malloc(8 * n); float* p1 = malloc(8 * n); uint8_t* mask = malloc(n);
        double tz = 1.0 + urand(&s), tx = 0.05 * (urand(&s) - 0.5), yaw = 0.02 * (urand(&s) - 0.5);
        for (int i = 0; i < n; ++i) {
            double X = (urand(&s) - 0.5) * 40, Y = (urand(&s) - 0.5) * 6, Z = 5 + urand(&s) * 60;
            double u0 = K[0] * X / Z + K[2], v0 = K[4] * Y / Z + K[5];
            double Xc = cos(yaw) * X - sin(yaw) * Z - tx, Zc = sin(yaw) * X + cos(yaw) * Z - tz;
            double u1 = K[0] * Xc / Zc + K[2], v1 = K[4] * Y / Zc + K[5];
            if (urand(&s) < outl) { u1 = urand(&s) * 1241; v1 = urand(&s) * 376; }
            p0[2*i] = (float)(u0 + 0.3 * (urand(&s) - 0.5)); p0[2*i+1] = (float)(v0 + 0.3 * (urand(&s) - 0.5));
            p1[2*i] = (float)(u1 + 0.3 * (urand(&s) - 0.5)); p1[2*i+1] = (float)(v1 + 0.3 * (urand(&s) - 0.5));
        }
        double E[9];
        int before = g_nco;
        int nm_; vo_o_find_essential(p0, p1, n, K, 0.999, 1.0, 1000, E, mask, &nm_);
        fprintf(stderr, "problem %d: %d hypotheses\n", pb, g_nco - before);
        free(p0); free(p1); free(mask);
    }
    int hist[302] = {0}, per[10] = {0}, lastcyc[302] = {0}, cyc = 0, conv = 0; long tot = 0, saved = 0;
    for (int k = 0; k < g_nco; ++k) {
        int pd, st; int sw = sweeps(g_co[k], &pd, &st);
        hist[sw]++; tot += sw;
        if (pd) { cyc++; per[pd < 10 ? pd : 9]++; lastcyc[st + pd < 301 ? st + pd : 300]++; saved += 300 - (st + pd); }
        if (sw < 300) conv++;
    }
    printf("hypotheses %d mean sweeps %.1f  converged(<300) %d  cycles found %d  sweeps saved by cycle jump %.1f per hyp\n",
           g_nco, (double)tot / g_nco, conv, cyc, (double)saved / g_nco);
    for (int p = 1; p < 10; ++p) if (per[p]) printf(" period %d: %d\n", p, per[p]);
    { int a2 = 0; for (int i = 0; i <= 300; ++i) { a2 += lastcyc[i]; if (lastcyc[i] && (i % 20 == 0)) printf("  cycle detected by sweep %d: %d\n", i, a2); } }
    int acc = 0; for (int i = 0; i <= 301; ++i) { acc += hist[i]; if (hist[i] && (i % 25 == 0 || i >= 295 || i < 30)) printf("  sweeps<=%d: %d\n", i, acc); }
    return 0;
}
