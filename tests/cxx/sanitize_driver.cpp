// Host sanitizer run (AddressSanitizer + UndefinedBehaviorSanitizer) over the CPU code this repo
// compiles for the host: the oracle's C restatement (oracle/*.c: every primitive the golden
// fixtures and the GPU parity tests rely on) and the PNG ingest (csrc/vo_ingest.cpp).  GPU
// code is not sanitizable on this pool (no GPU ASan / XNACK); the kernels are checked by the
// bit-exact parity tests instead.  Built and run by tests/test_sanitizers.py; exits non-zero
// (the sanitizers abort) on any out-of-bounds access, use-after-free, leak or UB.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../oracle/vo_oracle.h"

extern "C" {
int vo_png_info(const uint8_t* data, size_t len, int* w, int* h, int* channels, int* depth);
int vo_png_decode_gray(const uint8_t* data, size_t len, uint8_t* out, int64_t pitch, int w, int h);
}

static float noise(float x, float y)
{
    // smooth value noise: bilinear blend of hashed lattice values, three octaves
    float v = 0.f, amp = 1.f, f = 1.f / 16.f;
    for (int o = 0; o < 3; ++o) {
        const float fx = x * f, fy = y * f;
        const int ix = (int)std::floor(fx), iy = (int)std::floor(fy);
        const float ax = fx - ix, ay = fy - iy;
        auto h = [&](int a, int b) {
            uint32_t k = (uint32_t)a * 73856093u ^ (uint32_t)b * 19349663u ^ (uint32_t)o * 83492791u;
            k ^= k >> 13; k *= 0x5bd1e995u; k ^= k >> 15;
            return (float)(k & 1023) / 1023.f;
        };
        v += amp * ((1 - ax) * (1 - ay) * h(ix, iy) + ax * (1 - ay) * h(ix + 1, iy) + (1 - ax) * ay * h(ix, iy + 1) +
                    ax * ay * h(ix + 1, iy + 1));
        amp *= 0.5f;
        f *= 2.f;
    }
    return v;
}

#define CHECK(x) do { int rc_ = (x); if (rc_ < 0) { std::printf("FAIL %s rc=%d\n", #x, rc_); return 1; } } while (0)

int main(int argc, char** argv)
{
    const int W = 320, H = 240;
    std::vector<uint8_t> a(W * H), b(W * H);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            a[y * W + x] = (uint8_t)std::lrint(40 + 150 * noise((float)x, (float)y) / 1.75f);
            b[y * W + x] = (uint8_t)std::lrint(40 + 150 * noise(x - 1.3f, y - 0.7f) / 1.75f);
        }
    std::vector<uint8_t> half(((W + 1) / 2) * ((H + 1) / 2));
    CHECK(vo_o_pyrdown(a.data(), W, H, half.data()));
    std::vector<int16_t> der(2 * W * H);
    CHECK(vo_o_scharr(a.data(), W, H, der.data()));
    std::vector<float> eig(W * H);
    CHECK(vo_o_eigmap(a.data(), W, H, 3, 0, 0.04, eig.data()));
    CHECK(vo_o_eigmap(a.data(), W, H, 5, 1, 0.04, eig.data()));
    std::vector<float> corners(2 * 600);
    int nc = 0;
    CHECK(vo_o_gftt(a.data(), W, H, 600, 0.01, 5.0, 3, 0, 0.04, corners.data(), 600, &nc));
    std::vector<float> out(2 * nc);
    std::vector<uint8_t> st(nc);
    std::vector<float> err(nc);
    CHECK(vo_o_lk(a.data(), b.data(), W, H, corners.data(), nc, out.data(), st.data(), err.data(), 15, 15, 3, 3, 30, 0.01, 1e-4));
    CHECK(vo_o_lk(a.data(), b.data(), W, H, corners.data(), nc, out.data(), st.data(), err.data(), 21, 21, 5, 3, 50, 0.02, 1e-4));
    const int cap = 8192;
    std::vector<float> kp0(6 * cap), kp1(6 * cap), d0((size_t)128 * cap), d1((size_t)128 * cap);
    int n0 = 0, n1 = 0;
    CHECK(vo_o_sift(a.data(), W, H, kp0.data(), d0.data(), cap, &n0));
    CHECK(vo_o_sift_n(b.data(), W, H, 200, kp1.data(), d1.data(), cap, &n1));
    std::vector<int32_t> idx2(2 * (n0 > 0 ? n0 : 1));
    std::vector<float> dist2(2 * (n0 > 0 ? n0 : 1));
    CHECK(vo_o_bf_knn2(d0.data(), n0, d1.data(), n1, 128, idx2.data(), dist2.data()));
    std::vector<float> resp(1000);
    std::vector<int32_t> perm(1000);
    for (int i = 0; i < 1000; ++i) resp[i] = (float)((i * 7919) % 97) / 97.f;
    CHECK(vo_o_retain_best(resp.data(), 1000, 100, perm.data()));
    // two-view and PnP geometry on synthetic points
    const double K[9] = {500, 0, 160, 0, 500, 120, 0, 0, 1};
    const int n = 200;
    std::vector<float> X(3 * n), p0(2 * n), p1(2 * n);
    const double th = 0.02, tx = 0.3, tz = 1.0;
    for (int i = 0; i < n; ++i) {
        const double x = noise((float)i, 3.f) * 8 - 4, y = noise(5.f, (float)i) * 6 - 3, z = 6 + 20 * noise((float)i, (float)i);
        X[3 * i] = (float)x; X[3 * i + 1] = (float)y; X[3 * i + 2] = (float)z;
        p0[2 * i] = (float)(K[0] * x / z + K[2]); p0[2 * i + 1] = (float)(K[4] * y / z + K[5]);
        const double x2 = std::cos(th) * x + std::sin(th) * z + tx, z2 = -std::sin(th) * x + std::cos(th) * z + tz;
        p1[2 * i] = (float)(K[0] * x2 / z2 + K[2]) + (i % 17 == 0 ? 9.f : 0.f);
        p1[2 * i + 1] = (float)(K[4] * y / z2 + K[5]);
    }
    double E[9], R[9], t[3];
    std::vector<uint8_t> mask(n);
    int nm = 0, ng = 0;
    CHECK(vo_o_find_essential(p0.data(), p1.data(), n, K, 0.99, 1.0, 1000, E, mask.data(), &nm));
    CHECK(vo_o_recover_pose(E, p0.data(), p1.data(), n, K, R, t, mask.data(), &ng));
    double P1[12] = {K[0], 0, K[2], 0, 0, K[4], K[5], 0, 0, 0, 1, 0}, P2[12];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 4; ++c) {
            double s = 0;
            for (int k = 0; k < 3; ++k) s += K[3 * r + k] * (c < 3 ? R[3 * k + c] : t[k]);
            P2[4 * r + c] = s;
        }
    std::vector<float> X4(4 * n);
    CHECK(vo_o_triangulate(P1, P2, p0.data(), p1.data(), n, X4.data()));
    double rvec[3], tvec[3];
    std::vector<int32_t> inl(n);
    int ni = 0, ok = 0, it = 0;
    CHECK(vo_o_pnp_ransac_p3p(X.data(), p1.data(), n, K, 500, 8.0, 0.99, rvec, tvec, inl.data(), &ni, &ok, &it));
    CHECK(vo_o_rodrigues_v2m(rvec, R));
    CHECK(vo_o_rodrigues_m2v(R, rvec));
    // PNG ingest on the file the test wrote
    if (argc > 1) {
        FILE* f = std::fopen(argv[1], "rb");
        if (!f) { std::printf("FAIL open %s\n", argv[1]); return 1; }
        std::vector<uint8_t> buf;
        uint8_t tmp[4096];
        size_t m;
        while ((m = std::fread(tmp, 1, sizeof tmp, f)) > 0) buf.insert(buf.end(), tmp, tmp + m);
        std::fclose(f);
        int w = 0, h = 0, ch = 0, dp = 0;
        CHECK(vo_png_info(buf.data(), buf.size(), &w, &h, &ch, &dp));
        std::vector<uint8_t> img((size_t)w * h);
        CHECK(vo_png_decode_gray(buf.data(), buf.size(), img.data(), w, w, h));
        // a truncated file must fail cleanly, not read past the buffer
        if (vo_png_decode_gray(buf.data(), buf.size() / 2, img.data(), w, w, h) >= 0) { std::printf("FAIL truncated\n"); return 1; }
    }
    std::printf("ok corners=%d sift=%d/%d essential_inliers=%d pnp_inliers=%d\n", nc, n0, n1, ng, ni);
    return 0;
}
