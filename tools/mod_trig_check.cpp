// tools/mod_trig_check.cpp — mod_trig (util.rs:3-6: x - TWO_PI * floor(x / TWO_PI), IEEE f32
// division) against the device's division-free form (modem_device.h phase_from_f: q0 = x * RC,
// r = fma(-q0, TWO_PI, x), q1 = fma(r, RC, q0), floor(q1)) for every finite f32 input, negative
// ones included: the same result, bitwise, once -0 is mapped to +0 (x + 0.0f; without it -0 alone
// differs: the reference gives +0, the division-free form -0). Decides whether the scanned phasors'
// recurrence (tx_scan: DMPSK / MFSK / BFSK, whose phases can be negative) may use the fast form.
// Build: g++ -O2 -std=c++17 -ffp-contract=off -pthread tools/mod_trig_check.cpp -o /tmp/mod_trig_check
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

int main(int argc, char** argv) {
    const int nt = argc > 1 ? std::atoi(argv[1]) : 8;
    const float TWO_PI = 0x1.921fb6p+2f, RC = 0x1.45f306p-3f;
    std::atomic<uint64_t> bad{0}, checked{0};
    std::atomic<uint64_t> first{~0ull};
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            uint64_t b = 0, n = 0;
            for (uint64_t u = (uint64_t)t; u < (1ull << 32); u += (uint64_t)nt) {
                const uint32_t w = (uint32_t)u;
                float x;
                std::memcpy(&x, &w, 4);
                if (!std::isfinite(x)) continue;
                ++n;
                const float fr = std::floor(x / TWO_PI);
                const float xz = x + 0.0f;             // -0 -> +0 (the only input that differed)
                const float q0 = xz * RC;
                const float r = std::fma(-q0, TWO_PI, xz);
                const float q1 = std::fma(r, RC, q0);
                const float ff = std::floor(q1);
                const float a = x - TWO_PI * fr, c = xz - TWO_PI * ff;
                uint32_t ua, uc;
                std::memcpy(&ua, &a, 4);
                std::memcpy(&uc, &c, 4);
                if (ua != uc && !(std::isnan(a) && std::isnan(c))) {
                    ++b;
                    uint64_t f = first.load();
                    while (u < f && !first.compare_exchange_weak(f, u)) {}
                }
            }
            bad += b;
            checked += n;
        });
    for (auto& x : th) x.join();
    std::printf("mod_trig fast form: %llu finite inputs, %llu mismatches", (unsigned long long)checked.load(),
                (unsigned long long)bad.load());
    if (bad.load()) {
        const uint32_t w = (uint32_t)first.load();
        float x;
        std::memcpy(&x, &w, 4);
        std::printf(" (first 0x%08x = %a)", w, x);
    }
    std::printf("\n");
    return bad.load() ? 1 : 0;
}
