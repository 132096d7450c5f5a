#include <stdio.h>
#include <string.h>
#include <math.h>
#include <float.h>
#include <stdint.h>
#include <stdlib.h>
static double g_co[200000][11]; static int g_nco = 0;
static void sp_hook(const double* c) { if (g_nco < 200000) { memcpy(g_co[g_nco], c, 11 * sizeof(double)); g_nco++; } }
#include "geom_hooked.c"
/* serial reference = oracle's solve_poly; pipelined emulation of five_point_grp's schedule */
static void pipelined(const double* c, cplx* out)
{
    cplx co[11], r[10];
    for (int i = 0; i <= 10; ++i) { co[i].re = c[i]; co[i].im = 0; }
    cplx p = {1, 0}, rr = {1, 1};
    for (int i = 0; i < 10; ++i) { r[i] = p; p = c_mul(p, rr); }
    for (int iter = 0; iter < 300; ++iter) {
        cplx pm[10], num[10], den[10];
        for (int li = 0; li < 10; ++li) {
            pm[li] = r[li]; num[li] = co[10]; den[li] = co[10];
            for (int j = 0; j < 10; ++j) num[li] = c_add(c_mul(num[li], pm[li]), co[10 - j - 1]);
        }
        double maxDiff = 0;
        for (int t = 0; t < 10; ++t) {
            int li = t;
            for (int j = t + 1; j < 10; ++j) { cplx d = c_sub(pm[li], r[j]); if (!(d.re == 0 && d.im == 0)) den[li] = c_mul(den[li], d); }
            cplx q = c_div(num[li], den[li]);
            cplx nr = c_sub(pm[li], q);
            double a = sqrt(q.re * q.re + q.im * q.im);
            r[t] = nr;
            if (a > maxDiff) maxDiff = a;
            for (int l2 = t + 1; l2 < 10; ++l2) { cplx d = c_sub(pm[l2], r[t]); if (!(d.re == 0 && d.im == 0)) den[l2] = c_mul(den[l2], d); }
        }
        if (maxDiff <= 0) break;
    }
    for (int i = 0; i < 10; ++i) { if (fabs(r[i].im) < 1e-100) r[i].im = 0; out[i] = r[i]; }
}
static double urand(uint64_t* s) { *s = *s * 6364136223846793005ULL + 1442695040888963407ULL; return (double)(*s >> 11) / 9007199254740992.0; }
int main(void)
{
    uint64_t s = 777;
    const double K[9] = {718.856, 0, 607.1928, 0, 718.856, 185.2157, 0, 0, 1};
    for (int pb = 0; pb < 20; ++pb) {
        int n = 800; float* p0 = malloc(8 * n); float* p1 = malloc(8 * n); uint8_t* mask = malloc(n);
        for (int i = 0; i < n; ++i) {
            double X = (urand(&s) - 0.5) * 40, Y = (urand(&s) - 0.5) * 6, Z = 5 + urand(&s) * 60;
            p0[2*i] = (float)(K[0] * X / Z + K[2]); p0[2*i+1] = (float)(K[4] * Y / Z + K[5]);
            double Zc = Z - 1.3, Xc = X - 0.02;
            p1[2*i] = (float)(K[0] * Xc / Zc + K[2] + 0.3 * (urand(&s) - 0.5)); p1[2*i+1] = (float)(K[4] * Y / Zc + K[5]);
            if (urand(&s) < 0.4) { p1[2*i] = urand(&s) * 1241; p1[2*i+1] = urand(&s) * 376; }
        }
        double E[9]; int nm_;
        vo_o_find_essential(p0, p1, n, K, 0.999, 1.0, 1000, E, mask, &nm_);
        free(p0); free(p1); free(mask);
    }
    int bad = 0;
    for (int k = 0; k < g_nco; ++k) {
        cplx a[10], b[10];
        solve_poly(g_co[k], 10, a);
        pipelined(g_co[k], b);
        if (memcmp(a, b, sizeof a)) ++bad;
    }
    printf("polynomials %d, pipelined != serial: %d\n", g_nco, bad);
    return 0;
}
