// Test harness (CPU only): OpenCV 4.6 KeyPointsFilter::retainBest (features2d/src/
// keypoint.cpp) written with the real std::nth_element / std::partition of this image's
// libstdc++, on (response, index) records.  tests/test_retain_best.py compares the order
// it leaves with the oracle's step-for-step restatement (oracle/vo_oracle_sift.c) and the
// GPU kernel (k_sift_retain_best).
//
//   retain_best_std select   stdin: n n_points, n responses (hex floats)
//                            stdout: kept, then the n record indices in final order
//   retain_best_std killer n n_points
//                            stdout: n responses on which std::nth_element exhausts its
//                            depth limit (McIlroy's adversary), so the __heap_select
//                            fallback is exercised
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

struct Rec {
    float response;
    int index;
};

static size_t retain_best(std::vector<Rec>& kp, int n_points)
{
    if (n_points < 0 || kp.size() <= (size_t)n_points) return kp.size();
    if (n_points == 0) return 0;
    std::nth_element(kp.begin(), kp.begin() + n_points - 1, kp.end(),
                     [](const Rec& a, const Rec& b) { return a.response > b.response; });
    const float amb = kp[n_points - 1].response;
    auto ne = std::partition(kp.begin() + n_points, kp.end(), [amb](const Rec& r) { return r.response >= amb; });
    return (size_t)(ne - kp.begin());
}

// McIlroy, "A killer adversary for quicksort" (1999): values are fixed lazily so that every
// partition step peels off as few elements as possible.
static std::vector<int> g_val;
static int g_gas, g_solid, g_cand;

static bool adv_greater(int x, int y)
{
    if (g_val[x] == g_gas && g_val[y] == g_gas) {
        if (x == g_cand) g_val[x] = g_solid++;
        else g_val[y] = g_solid++;
    }
    if (g_val[x] == g_gas) g_cand = x;
    else if (g_val[y] == g_gas) g_cand = y;
    return g_val[x] < g_val[y];          // "x's response is greater" <=> smaller value
}

int main(int argc, char** argv)
{
    if (argc >= 4 && !std::strcmp(argv[1], "killer")) {
        const int n = std::atoi(argv[2]), n_points = std::atoi(argv[3]);
        g_gas = n;
        g_solid = 0;
        g_cand = -1;
        g_val.assign(n, n);
        std::vector<int> ix(n);
        for (int i = 0; i < n; ++i) ix[i] = i;
        std::nth_element(ix.begin(), ix.begin() + n_points - 1, ix.end(), adv_greater);
        for (int i = 0; i < n; ++i) std::printf("%a\n", (float)(n - g_val[i]));
        return 0;
    }
    int n = 0, n_points = 0;
    if (std::scanf("%d %d", &n, &n_points) != 2) return 1;
    std::vector<Rec> kp(n);
    for (int i = 0; i < n; ++i) {
        if (std::scanf("%a", &kp[i].response) != 1) return 1;
        kp[i].index = i;
    }
    const size_t kept = retain_best(kp, n_points);
    std::printf("%zu\n", kept);
    for (int i = 0; i < n; ++i) std::printf("%d\n", kp[i].index);
    return 0;
}
