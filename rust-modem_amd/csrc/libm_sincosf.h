// rust-modem_amd/csrc/libm_sincosf.h — f32 sin / cos with the exact results of the host libm
// the reference calls (Rust's f32::sin / f32::cos lower to sinf / cosf; on x86_64 Linux that
// is glibc 2.35, whose implementation is the "optimized-routines" algorithm: double-precision
// evaluation after a range reduction, sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, sincosf.h).
// The algorithm is restated here from its published description, with the constants it uses
// (read from this image's libm: __sincosf_table, __inv_pio4); FMA selects the build glibc runs
// on x86-64 hosts with FMA (its ifunc picks the -mfma variant, in which GCC contracts every
// a + b*c of the polynomials and the reduction into one fused operation).
//
// Compiled by hipcc (device code: the bit-exact demodulator, mix MODEM_MIX_REFERENCE_REAL_EXACT)
// and by gcc (tools/libm_check.c compares it with the host's sinf / cosf for every float).
// Every operation is explicit (no contraction left to the compiler).
//
// Attribution: the algorithm and its constants (the polynomial coefficients of sincos_t and the
// 4/pi bit table __inv_pio4) are those of ARM's optimized-routines single-precision sinf/cosf
// (Szabolcs Nagy, Arm Ltd., 2018), as contributed to and shipped in the GNU C Library
// (sysdeps/ieee754/flt-32/{s_sinf.c, s_cosf.c, sincosf.h, sincosf_poly.h}; glibc 2.35). In
// glibc those files are distributed under the GNU Lesser General Public License v2.1 or later;
// optimized-routines itself is available under the MIT OR Apache-2.0 WITH LLVM-exception
// licenses. This file restates that published algorithm for the device; no glibc source text
// is copied. The numeric constants are facts of the reference platform's libm that bit-exact
// parity with Rust's f32::sin / f32::cos on it requires.
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define LM_HD __host__ __device__ __forceinline__
#else
#define LM_HD static inline
#endif

namespace lm {

struct SinCosT {              // glibc's sincos_t, in its memory order
    double sign[4], hpi_inv, hpi, c0, c1, s1, c2, s2, c3, s3, c4;
};

// [0]: the table; [1]: the same with the cosine polynomial negated (quadrants 2, 3)
#define LM_TABLE(NEG)                                                                         \
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0, NEG 0x1.0p+0,       \
     NEG -0x1.ffffffd0c621cp-2, -0x1.555545995a603p-3, NEG 0x1.55553e1068f19p-5,              \
     0x1.1107605230bc4p-7, NEG -0x1.6c087e89a359dp-10, -0x1.994eb3774cf24p-13,                \
     NEG 0x1.99343027bf8c3p-16}

LM_HD uint32_t as_u32(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
LM_HD uint32_t abstop12(float x) { return (as_u32(x) >> 20) & 0x7ff; }

template <bool FMA> LM_HD double madd(double a, double b, double c) {   // a * b + c
#pragma clang fp contract(off)
    return FMA ? __builtin_fma(a, b, c) : a * b + c;
}

// The sine (n even) or cosine (n odd) polynomial of reduced x, x2 = x * x.
template <bool FMA> LM_HD float poly(double x, double x2, const SinCosT& p, int n) {
#pragma clang fp contract(off)
    if ((n & 1) == 0) {
        const double x3 = x * x2;
        const double s1 = madd<FMA>(x2, p.s3, p.s2);
        const double x7 = x3 * x2;
        const double s = madd<FMA>(x3, p.s1, x);
        return (float)madd<FMA>(x7, s1, s);
    }
    const double x4 = x2 * x2;
    const double c2 = madd<FMA>(x2, p.c4, p.c3);
    const double c1 = madd<FMA>(x2, p.c1, p.c0);
    const double x6 = x4 * x2;
    const double c = madd<FMA>(x4, p.c2, c1);
    return (float)madd<FMA>(x6, c2, c);
}

// |x| < 120: one multiply-subtract with the quadrant from a scaled float -> int conversion.
template <bool FMA> LM_HD double reduce_fast(double x, const SinCosT& p, int* np) {
#pragma clang fp contract(off)
    const double r = x * p.hpi_inv;
    const int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return madd<FMA>(-(double)n, p.hpi, x);
}

// Larger |x|: 4/pi to 192 bits, a 32 x 96 -> 128-bit multiply.
LM_HD double reduce_large(uint32_t xi, int* np) {
    // __inv_pio4[i]: bits 8i-24 .. 8i+8 of 2/pi's fraction (0xa2f9836e...), windows of a byte
    const uint8_t d[27] = {0, 0, 0, 0xa2, 0xf9, 0x83, 0x6e, 0x4e, 0x44, 0x15, 0x29, 0xfc, 0x27, 0x57,
                           0xd1, 0xf5, 0x34, 0xdd, 0xc0, 0xdb, 0x62, 0x95, 0x99, 0x3c, 0x43, 0x90, 0x41};
    const int i0 = (int)((xi >> 26) & 15);
    uint32_t a[3];
    for (int k = 0; k < 3; ++k) {
        const int i = i0 + 4 * k;
        a[k] = (uint32_t)d[i] << 24 | (uint32_t)d[i + 1] << 16 | (uint32_t)d[i + 2] << 8 | d[i + 3];
    }
    const int shift = (int)((xi >> 23) & 7);
    uint32_t m = (xi & 0xffffff) | 0x800000;
    m <<= shift;
    uint64_t res0 = (uint64_t)(m * a[0]);
    const uint64_t res1 = (uint64_t)m * a[1];
    const uint64_t res2 = (uint64_t)m * a[2];
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    const uint64_t n = (res0 + (1ULL << 61)) >> 62;
    res0 -= n << 62;
    *np = (int)n;
    return (double)(int64_t)res0 * 0x1.921fb54442d18p-62;     // pi63 = 2 pi * 2^-64
}

template <bool FMA> LM_HD float sinf(float y) {
#pragma clang fp contract(off)
    const SinCosT t0 = LM_TABLE(+), t1 = LM_TABLE(-);
    double x = y;
    int n;
    if (abstop12(y) < abstop12(0x1.921fb6p-1f)) {              // |y| < pi/4
        if (abstop12(y) < abstop12(0x1p-12f)) return y;
        return poly<FMA>(x, x * x, t0, 0);
    }
    if (abstop12(y) < abstop12(120.0f)) {
        x = reduce_fast<FMA>(x, t0, &n);
        const double s = t0.sign[n & 3];
        return poly<FMA>(x * s, x * x, (n & 2) ? t1 : t0, n);
    }
    if (abstop12(y) < abstop12(__builtin_inff())) {
        const uint32_t xi = as_u32(y);
        const int sign = (int)(xi >> 31);
        x = reduce_large(xi, &n);
        const double s = t0.sign[(n + sign) & 3];
        return poly<FMA>(x * s, x * x, ((n + sign) & 2) ? t1 : t0, n);
    }
    return (y - y) / (y - y);                                  // NaN (invalid) for inf / NaN
}

template <bool FMA> LM_HD float cosf(float y) {
#pragma clang fp contract(off)
    const SinCosT t0 = LM_TABLE(+), t1 = LM_TABLE(-);
    double x = y;
    int n;
    if (abstop12(y) < abstop12(0x1.921fb6p-1f)) {
        if (abstop12(y) < abstop12(0x1p-12f)) return 1.0f;
        return poly<FMA>(x, x * x, t0, 1);
    }
    if (abstop12(y) < abstop12(120.0f)) {
        x = reduce_fast<FMA>(x, t0, &n);
        const double s = t0.sign[n & 3];
        return poly<FMA>(x * s, x * x, (n & 2) ? t1 : t0, n ^ 1);
    }
    if (abstop12(y) < abstop12(__builtin_inff())) {
        const uint32_t xi = as_u32(y);
        const int sign = (int)(xi >> 31);
        x = reduce_large(xi, &n);
        const double s = t0.sign[(n + sign) & 3];
        return poly<FMA>(x * s, x * x, ((n + sign) & 2) ? t1 : t0, n ^ 1);
    }
    return (y - y) / (y - y);
}

}  // namespace lm
