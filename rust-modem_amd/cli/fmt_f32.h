// rust-modem_amd/cli/fmt_f32.h — Rust's `Display` for f32 (what `println!("{}", x)` prints):
// the shortest digit string that reads back to the same f32 (the closest one on ties), laid
// out positionally — padded with zeros, never an exponent, no trailing ".0" — with "-" on
// negatives including -0, "inf" / "-inf", "NaN". The digits come from std::to_chars in its
// shortest scientific form (fixed form would print large values exactly, e.g. 1e20f as
// 100000002004087734272, where Rust prints 100000000000000000000).
#pragma once
#include <charconv>
#include <cmath>
#include <cstdlib>
#include <cstring>

// Writes at most 64 chars to buf, returns the length.
inline int fmt_f32(char* buf, float v) {
    if (std::isnan(v)) { std::memcpy(buf, "NaN", 3); return 3; }
    if (std::isinf(v)) {
        if (v > 0) { std::memcpy(buf, "inf", 3); return 3; }
        std::memcpy(buf, "-inf", 4);
        return 4;
    }
    char t[48];
    const std::to_chars_result r = std::to_chars(t, t + sizeof t, v, std::chars_format::scientific);
    *r.ptr = 0;
    const char* s = t;
    int n = 0;
    if (*s == '-') { buf[n++] = '-'; ++s; }
    char dig[16];                                    // d.ddd -> dddd
    int nd = 0;
    for (; *s && *s != 'e'; ++s)
        if (*s != '.') dig[nd++] = *s;
    const int e = std::atoi(s + 1);                  // value = d.ddd x 10^e
    const int p = e + 1;                             // digits before the point
    if (p <= 0) {
        buf[n++] = '0';
        buf[n++] = '.';
        for (int i = 0; i < -p; ++i) buf[n++] = '0';
        for (int i = 0; i < nd; ++i) buf[n++] = dig[i];
    } else if (p >= nd) {
        for (int i = 0; i < nd; ++i) buf[n++] = dig[i];
        for (int i = nd; i < p; ++i) buf[n++] = '0';
    } else {
        for (int i = 0; i < p; ++i) buf[n++] = dig[i];
        buf[n++] = '.';
        for (int i = p; i < nd; ++i) buf[n++] = dig[i];
    }
    return n;
}
