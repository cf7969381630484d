// Host check of aten_inner_sum's fast path for 8..15 elements (dfq_common.h)
// against the generic walk it replaces (the tail, then 8 aten_row_sum streams),
// bit for bit, on random values mixed with -0, +-inf, NaN, denormals and huge
// values.  Built and run by tests/test_inner_sum_fast_path.py (no GPU).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>

#include "dfq_common.h"

static uint32_t bits(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}

int main() {
    std::mt19937 rng(12345);
    std::uniform_real_distribution<float> uni(-1.f, 1.f);
    const float special[] = {-0.f, 0.f, INFINITY, -INFINITY, NAN, 1e-40f, -1e-40f, 3e38f, -3e38f, 1.f, -1.f};
    long checked = 0, bad = 0;
    for (int trial = 0; trial < 200000; ++trial) {
        const int n = 8 + trial % 8;
        float x[16];
        for (int i = 0; i < n; ++i) {
            const int r = (int)(rng() % 8);
            x[i] = r == 0 ? special[rng() % (sizeof(special) / sizeof(float))] : uni(rng) * std::ldexp(1.f, (int)(rng() % 40) - 20);
        }
        auto get = [&](int64_t i) { return x[i]; };
        const float fast = dfq::aten_inner_sum(get, n);
        // the generic walk (vs = 1)
        float fa = 0.f;
        for (int64_t k = 8; k < n; ++k) fa += get(k);
        for (int l = 0; l < 8; ++l) fa += dfq::aten_row_sum([&](int64_t i) { return get(8 * i + l); }, 1);
        ++checked;
        const bool same = bits(fast) == bits(fa) || (std::isnan(fast) && std::isnan(fa));
        if (!same && bad++ < 5) std::printf("MISMATCH n=%d fast=%a generic=%a\n", n, fast, fa);
    }
    std::printf("checked %ld mismatches %ld\n", checked, bad);
    return bad ? 1 : 0;
}
