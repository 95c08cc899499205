// tools/libm_check.cpp — every f32 input through rust-modem_amd/csrc/libm_sincosf.h against the
// host libm's sinf / cosf (bitwise; NaN == NaN), for the FMA and the plain build of the
// algorithm. Usage: tools/libm_check [threads] [stride]  (stride 1 = all 2^32 inputs).
// Build: g++ -O2 -std=c++17 -ffp-contract=off -Wno-unknown-pragmas -pthread tools/libm_check.cpp -o ...
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "../rust-modem_amd/csrc/libm_sincosf.h"

static bool same(float a, float b) {
    if (std::isnan(a) && std::isnan(b)) return true;
    return lm::as_u32(a) == lm::as_u32(b);
}

int main(int argc, char** argv) {
    const int nt = argc > 1 ? std::atoi(argv[1]) : 8;
    const uint64_t stride = argc > 2 ? std::strtoull(argv[2], nullptr, 0) : 1;
    std::atomic<uint64_t> bad[4] = {0, 0, 0, 0};
    std::atomic<uint64_t> first[4];
    for (auto& f : first) f = ~0ull;
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            uint64_t b[4] = {0, 0, 0, 0};
            for (uint64_t u = (uint64_t)t * stride; u < (1ull << 32); u += (uint64_t)nt * stride) {
                float x;
                const uint32_t v = (uint32_t)u;
                memcpy(&x, &v, 4);
                const float s = ::sinf(x), c = ::cosf(x);
                const bool r[4] = {same(lm::sinf<true>(x), s), same(lm::cosf<true>(x), c),
                                   same(lm::sinf<false>(x), s), same(lm::cosf<false>(x), c)};
                for (int k = 0; k < 4; ++k)
                    if (!r[k]) {
                        ++b[k];
                        uint64_t f = first[k];
                        while (u < f && !first[k].compare_exchange_weak(f, u)) {}
                    }
            }
            for (int k = 0; k < 4; ++k) bad[k] += b[k];
        });
    for (auto& x : th) x.join();
    const char* name[4] = {"sinf fma", "cosf fma", "sinf plain", "cosf plain"};
    for (int k = 0; k < 4; ++k)
        std::printf("%-11s mismatches %llu (first 0x%08llx)\n", name[k], (unsigned long long)bad[k],
                    (unsigned long long)(first[k].load() == ~0ull ? 0 : first[k].load()));
    return bad[0] == 0 && bad[1] == 0 ? 0 : 1;
}
