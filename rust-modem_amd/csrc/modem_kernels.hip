// rust-modem_amd/csrc/modem_kernels.hip — gfx950 kernels for the modem sample path.
//
// TX  (modulator.rs:64-101 + fir.rs:18-34 + modulator.rs:45-48)
//   tx_fast<SPS>: one workgroup = TS = 256*R symbols.
//     1. stage the TS + K - 1 symbols it needs (bits -> bytes_to_bits index -> LUT) in LDS
//        (digital/util.rs:5-11, the phasor's i()/q() as a precomputed table);
//     2. each lane computes R consecutive symbols x SPS phases of the zero-stuffed
//        polyphase FIR  y[m*SPS+p] = sum_t h[p+SPS*t] * a[m-t]  with a sliding register
//        window (one ds_read_b64 per R*SPS complex MACs; taps are wave-uniform s_loads);
//     3. transposes the tile through LDS and, per pair of consecutive samples, computes the
//        bit-exact carrier phase (carrier.rs:17-19, util.rs:3-6), mixes (i+jq)e^{j phase}
//        and writes 16-B coalesced stores.
// RX  (demodulator.rs:44-56 + fir.rs:18-34, evaluated only at the kept instants)
//   rx_fast<DEC>: one workgroup = TS = 256*R output symbols.
//     1. streams the (TS+K-1)*DEC input samples it needs with 16-B loads, applies the
//        conjugate (or the reference's real) mix per sample and scatters them into DEC
//        polyphase planes in LDS  z_b[m] = z[m*DEC + D - b];
//     2. each lane computes R consecutive outputs  r_k = sum_b sum_t h[b+DEC*t] z_b[k-t]
//        with one sliding window per plane (ds_read_b64 per R complex MACs);
//     3. hard decision + store.
// Both kernels fold the streaming-state update (filter history, leftover bits) into
// workgroup 0, writing the *other* half of a double buffer, so a call is one launch.
#include "modem_internal.h"

#include <hip/hip_fp16.h>

#include <map>
#include <mutex>
#include <utility>

namespace mk {

// ----------------------------------------------------------------------------------------
// Bit-exact reference carrier phase: mod_trig(w * (n as f32)).
//   x = fl(w * fl(n)); phase = fl(x - fl(TWO_PI * floor(fl(x / TWO_PI)))).
// fl(x / TWO_PI) is replaced by q1 = q0 + r*RC (q0 = x*RC, r = fma(-q0, TWO_PI, x)):
// q1 differs from the IEEE quotient for some x but floor(q1) == floor(fl(x/TWO_PI)) for
// every non-negative finite f32 (checked exhaustively on the host: tests/test_phase_math.py),
// so the phase is bit-identical. contract(off) keeps TWO_PI*f and the subtraction
// separately rounded, as rustc does.
constexpr float kTwoPi = 0x1.921fb6p+2f;   // std::f32::consts::PI * 2.0 (0x40c90fdb)
constexpr float kRcp2Pi = 0x1.45f306p-3f;  // fl(1 / kTwoPi)

__device__ __forceinline__ float phase_from_f(float w, float nf) {
#pragma clang fp contract(off)
    const float x = w * nf;
    const float q0 = x * kRcp2Pi;
    const float r = __builtin_fmaf(-q0, kTwoPi, x);
    const float q1 = __builtin_fmaf(r, kRcp2Pi, q0);
    const float f = __builtin_floorf(q1);
    const float p = kTwoPi * f;
    return x - p;
}

// `n as f32` with round-to-nearest-even: one v_cvt_f32_u32 below 2^32, the compiler's
// exact u64 -> f32 sequence above.
__device__ __forceinline__ float carrier_phase(float w, uint64_t n, bool small_n) {
    const float nf = small_n ? (float)(uint32_t)n : (float)n;
    return phase_from_f(w, nf);
}

// Same, for n = base + off with a wave-uniform 64-bit base and a 32-bit lane offset.
__device__ __forceinline__ float carrier_phase_off(float w, uint64_t base, int off, bool small_n) {
    const float nf = small_n ? (float)((uint32_t)base + (uint32_t)off) : (float)(base + (int64_t)off);
    return phase_from_f(w, nf);
}

// sin/cos of a phase in [0, 2pi]. MODEM_PRECISE_TRIG selects a Cody-Waite + minimax
// polynomial (<= 2 ulp); the default uses the hardware v_sin_f32/v_cos_f32 (input in
// revolutions). Either way the sample tolerance is set in tests/test_gpu_parity.py.
__device__ __forceinline__ void sincos_phase(float ph, float& s, float& c) {
#if defined(MODEM_ABLATE_TRIG)        // profiling builds only (tools/ablate.sh)
    s = ph; c = 1.0f;
    return;
#endif
#ifdef MODEM_PRECISE_TRIG
    const float j = __builtin_rintf(ph * 0.63661977236758134f);
    float r = __builtin_fmaf(-j, 1.57079637050628662f, ph);
    r = __builtin_fmaf(-j, -4.37113900018624283e-8f, r);
    const float r2 = r * r;
    float sp = __builtin_fmaf(r2, -1.9515295891e-4f, 8.3321608736e-3f);
    sp = __builtin_fmaf(r2, sp, -1.6666654611e-1f);
    const float sr = __builtin_fmaf(r * r2, sp, r);
    float cp = __builtin_fmaf(r2, 2.443315711809948e-5f, -1.388731625493765e-3f);
    cp = __builtin_fmaf(r2, cp, 4.166664568298827e-2f);
    const float cr = __builtin_fmaf(r2 * r2, cp, __builtin_fmaf(-0.5f, r2, 1.0f));
    const int q = (int)j & 3;
    const float ss = (q & 1) ? cr : sr, cc = (q & 1) ? sr : cr;
    s = (q & 2) ? -ss : ss;
    c = ((q + 1) & 2) ? -cc : cc;
#else
    s = __sinf(ph);
    c = __cosf(ph);
#endif
}

typedef const __attribute__((address_space(4))) float cfloat;   // wave-uniform -> s_load
// (re, im) pair: one v_pk_fma_f32 per complex x real MAC, tap broadcast from an SGPR.
typedef float cf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ cf2 ldc(const float2* p) { return *reinterpret_cast<const cf2*>(p); }
__device__ __forceinline__ cf2 cmac(cf2 x, float h, cf2 acc) {
    return __builtin_elementwise_fma(x, (cf2){h, h}, acc);
}

// ---------------------------------------------------------------- symbol mapping (TX) ----
// bytes_to_bits (digital/util.rs:5-11) of symbol m's bits, MSB first, `b & 1` per byte.
__device__ __forceinline__ uint32_t tx_symbol_index(const TxParams& p, int64_t m) {
    const int bps = p.bps;
    if (p.fast_bits) {
        const uint8_t* b = p.bits + m * bps;
        if (bps == 4) {
            const uint32_t v = *reinterpret_cast<const uint32_t*>(b);
            return ((v & 1u) << 3) | ((v >> 6) & 4u) | ((v >> 15) & 2u) | ((v >> 24) & 1u);
        }
        if (bps == 2) {
            const uint32_t v = *reinterpret_cast<const uint16_t*>(b);
            return ((v & 1u) << 1) | ((v >> 8) & 1u);
        }
        if (bps == 1) return b[0] & 1u;
        if (bps == 8) {
            const uint64_t v = *reinterpret_cast<const uint64_t*>(b);
            uint32_t idx = 0;
#pragma unroll
            for (int q = 0; q < 8; ++q) idx |= (uint32_t)((v >> (8 * q)) & 1u) << (7 - q);
            return idx;
        }
    }
    uint32_t idx = 0;
    const int64_t l0 = m * bps;
    for (int q = 0; q < bps; ++q) {
        const int64_t l = l0 + q;   // logical bit position in [carry | bits]
        const uint8_t b = l < p.ncarry ? p.carry[l] : p.bits[l - p.ncarry];
        idx = (idx << 1) | (b & 1u);
    }
    return idx;
}

__device__ __forceinline__ float2 tx_symbol_value(const TxParams& p, int64_t m) {
    if (m < 0) return m >= -(int64_t)(p.K - 1) ? p.hist[m + p.K - 1] : make_float2(0.f, 0.f);
    if (m >= p.nsym_valid) return make_float2(0.f, 0.f);
    return p.lut[tx_symbol_index(p, m)];
}

// Streaming state for the next call, written by workgroup 0 into the other buffers.
__device__ void tx_state_update(const TxParams& p) {
    for (int i = threadIdx.x; i < p.K - 1; i += blockDim.x)
        p.hist_new[i] = tx_symbol_value(p, p.nsym - (p.K - 1) + i);
    if (p.update_carry) {
        for (int i = threadIdx.x; i < p.ncarry_new; i += blockDim.x) {
            const int64_t l = p.nsym * p.bps + i;
            p.carry_new[i] = l < p.ncarry ? p.carry[l] : p.bits[l - p.ncarry];
        }
    }
}

template <typename OutT> struct OutIO;
template <> struct OutIO<float> {
    __device__ static void store_pair(void* out, int64_t j, float a, float b, float c, float d) {
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + 2 * j) = make_float4(a, b, c, d);
    }
    __device__ static void store_one(void* out, int64_t j, float a, float b) {
        *reinterpret_cast<float2*>(reinterpret_cast<float*>(out) + 2 * j) = make_float2(a, b);
    }
    __device__ static void store_real_pair(void* out, int64_t j, float a, float b) {
        *reinterpret_cast<float2*>(reinterpret_cast<float*>(out) + j) = make_float2(a, b);
    }
    __device__ static void store_real_one(void* out, int64_t j, float a) {
        reinterpret_cast<float*>(out)[j] = a;
    }
};
template <> struct OutIO<__half> {
    __device__ static void store_pair(void* out, int64_t j, float a, float b, float c, float d) {
        const __half2 h0 = __floats2half2_rn(a, b), h1 = __floats2half2_rn(c, d);
        uint2 u;
        u.x = *reinterpret_cast<const uint32_t*>(&h0);
        u.y = *reinterpret_cast<const uint32_t*>(&h1);
        *reinterpret_cast<uint2*>(reinterpret_cast<__half*>(out) + 2 * j) = u;
    }
    __device__ static void store_one(void* out, int64_t j, float a, float b) {
        *reinterpret_cast<__half2*>(reinterpret_cast<__half*>(out) + 2 * j) = __floats2half2_rn(a, b);
    }
    __device__ static void store_real_pair(void* out, int64_t j, float a, float b) {
        *reinterpret_cast<__half2*>(reinterpret_cast<__half*>(out) + j) = __floats2half2_rn(a, b);
    }
    __device__ static void store_real_one(void* out, int64_t j, float a) {
        reinterpret_cast<__half*>(out)[j] = __float2half_rn(a);
    }
};

enum { OUT_IQ_MIXED = 0, OUT_IQ_BASEBAND = 1, OUT_REAL = 2 };

// Mix one filtered baseband sample onto the carrier (IQSample::modulate, modulator.rs:45-48).
template <int OUT_MODE>
__device__ __forceinline__ float2 tx_mix(float w, uint64_t n, bool small_n, float2 y) {
    if (OUT_MODE == OUT_IQ_BASEBAND) return y;
    float s, c;
    sincos_phase(carrier_phase(w, n, small_n), s, c);
    return make_float2(y.x * c - y.y * s, y.x * s + y.y * c);
}

template <int OUT_MODE, typename OutT>
__device__ __forceinline__ void tx_emit(const TxParams& p, int64_t j, float2 y0, float2 y1,
                                        bool two) {
    const uint64_t n = p.s0 + (uint64_t)j;
    const float2 z0 = tx_mix<OUT_MODE>(p.w, n, p.small_n, y0);
    if (two) {
        const float2 z1 = tx_mix<OUT_MODE>(p.w, n + 1, p.small_n, y1);
        if (OUT_MODE == OUT_REAL) OutIO<OutT>::store_real_pair(p.out, j, z0.x, z1.x);
        else OutIO<OutT>::store_pair(p.out, j, z0.x, z0.y, z1.x, z1.y);
    } else {
        if (OUT_MODE == OUT_REAL) OutIO<OutT>::store_real_one(p.out, j, z0.x);
        else OutIO<OutT>::store_one(p.out, j, z0.x, z0.y);
    }
}

// Same with the sample index split into a wave-uniform base and a 32-bit lane offset.
template <int OUT_MODE, typename OutT>
__device__ __forceinline__ void tx_emit_off(const TxParams& p, int64_t jb, int off, float2 y0, float2 y1,
                                            bool two) {
    const int64_t j = jb + off;
    float2 z0 = y0, z1 = y1;
#ifdef MODEM_ABLATE_MIX
    if (false) {
#else
    if (OUT_MODE != OUT_IQ_BASEBAND) {
#endif
        const uint64_t nb = p.s0 + (uint64_t)jb;
        float s, c;
        sincos_phase(carrier_phase_off(p.w, nb, off, p.small_n), s, c);
        z0 = make_float2(y0.x * c - y0.y * s, y0.x * s + y0.y * c);
        if (two) {
            sincos_phase(carrier_phase_off(p.w, nb, off + 1, p.small_n), s, c);
            z1 = make_float2(y1.x * c - y1.y * s, y1.x * s + y1.y * c);
        }
    }
    if (two) {
        if (OUT_MODE == OUT_REAL) OutIO<OutT>::store_real_pair(p.out, j, z0.x, z1.x);
        else OutIO<OutT>::store_pair(p.out, j, z0.x, z0.y, z1.x, z1.y);
    } else {
        if (OUT_MODE == OUT_REAL) OutIO<OutT>::store_real_one(p.out, j, z0.x);
        else OutIO<OutT>::store_one(p.out, j, z0.x, z0.y);
    }
}

template <int SPS> struct TxCfg {
    // R consecutive symbols per lane (odd: conflict-free ds_read_b64 of the window) ->
    // R*SPS consecutive output samples per lane.
    static constexpr int R = SPS == 1 ? 5 : SPS == 2 ? 3 : 1;
    static constexpr int NT = 256;
    static constexpr int TS = NT * R;            // symbols per tile
    static constexpr int CH = 8;                 // taps steps unrolled per loop trip
    static constexpr int U = (TS + 64 + NT - 1) / NT;    // staging slots prefetched per lane
};

// Raw bits word of symbol m (fast path: one aligned 1/2/4/8-byte load; the caller only asks
// for symbols of this call, so the load is unconditional).
__device__ __forceinline__ uint64_t tx_load_word(const uint8_t* bits, int bps, int64_t m) {
    const uint8_t* b = bits + m * bps;
    switch (bps) {
    case 1: return *b;
    case 2: return *reinterpret_cast<const uint16_t*>(b);
    case 4: return *reinterpret_cast<const uint32_t*>(b);
    default: return *reinterpret_cast<const uint64_t*>(b);
    }
}

// bytes_to_bits (digital/util.rs:5-11) of a little-endian word holding bps bytes, branch-free:
// the LSB of byte i sits at bit 8i; one multiply moves it to bit 27-i (32-bit form) or 63-i
// (64-bit form) without carries (all partial-product bit positions are distinct).
__device__ __forceinline__ uint32_t word_index(uint64_t v, int bps) {
    if (bps <= 4) {
        const uint32_t b = (uint32_t)v & 0x01010101u;
        return ((b * 0x08040201u) >> 24) >> (4 - bps);
    }
    const uint64_t b = v & 0x0101010101010101ull;
    return (uint32_t)((b * 0x8040201008040201ull) >> 56) >> (8 - bps);
}

template <int SPS, int R, typename TP>
__device__ __forceinline__ void tx_mac(cf2 (&acc)[R][SPS], const cf2 (&win)[R], TP h) {
    float hv[SPS];
#pragma unroll
    for (int q = 0; q < SPS; ++q) hv[q] = h[q];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int q = 0; q < SPS; ++q) acc[r][q] = cmac(win[r], hv[q], acc[r][q]);
}

template <int R>
__device__ __forceinline__ void shift_in(cf2 (&win)[R], cf2 v) {
#pragma unroll
    for (int r = R - 1; r > 0; --r) win[r] = win[r - 1];
    win[0] = v;
}

template <int SPS, int OUT_MODE, typename OutT>
__global__ __launch_bounds__(256) void tx_fast(const TxParams p) {
    using C = TxCfg<SPS>;
    constexpr int R = C::R, NT = C::NT, TS = C::TS, CH = C::CH, U = C::U;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int tid = threadIdx.x;
    const int K = p.K;
    const int NE = TS + K - 1;                         // symbols staged per tile
    float2* lut_s = lds + ((TS + K + 2) & ~1);         // LUT after the symbol window
    if (blockIdx.x == 0) tx_state_update(p);
    for (int i = tid; i < (1 << p.bps); i += NT) lut_s[i] = p.lut[i];

    // Persistent workgroup: a balanced contiguous range of tiles.
    const int64_t ntiles = (p.nsym + TS - 1) / TS;
    const int64_t t0 = ntiles * blockIdx.x / gridDim.x, t1 = ntiles * (blockIdx.x + 1) / gridDim.x;
    // "inside": every staged symbol is a data symbol of this call and the prefetch ring
    // covers the window -> unconditional loads, no per-element cases.
    const bool pf = p.fast_bits && NE <= NT * U;        // workgroup-uniform
    auto inside = [&](int64_t m0) { return pf && m0 - (K - 1) >= 0 && m0 + TS <= p.nsym_valid; };
    uint64_t pre[U];
    auto prefetch = [&](int64_t m0) {
        const int64_t mb = m0 - (K - 1);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = tid + NT * u;
            pre[u] = tx_load_word(p.bits, p.bps, mb + (e < NE ? e : NE - 1));
        }
    };
    if (t0 < t1 && inside(t0 * TS)) prefetch(t0 * TS);
    __syncthreads();   // LUT visible

    cfloat* taps = (cfloat*)p.taps;
    for (int64_t t = t0; t < t1; ++t) {
        const int64_t m0 = t * TS;
        // 1. stage symbols m0-(K-1) .. m0+TS-1 -> lds[1 ..] (lds[0]: pad for the last shift-in)
        if (inside(m0)) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int e = tid + NT * u;
                if (e < NE) lds[1 + e] = lut_s[word_index(pre[u], p.bps)];
            }
        } else {   // first / last tiles, leftover bits, flush: one symbol at a time
            for (int e = tid; e < NE; e += NT) {
                const int64_t m = m0 - (K - 1) + e;
                lds[1 + e] = m < 0 ? p.hist[m + K - 1]
                                   : (m >= p.nsym_valid ? make_float2(0.f, 0.f) : lut_s[tx_symbol_index(p, m)]);
            }
        }
        __syncthreads();
        if (t + 1 < t1 && inside(m0 + TS)) prefetch(m0 + TS);   // next bits fly during the FIR

        // 2. polyphase FIR, R symbols x SPS phases per lane.
        cf2 acc[R][SPS];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int q = 0; q < SPS; ++q) acc[r][q] = (cf2){0.f, 0.f};
        const float2* base = lds + 1 + tid * R + (K - 1);   // base[j] = a[m0 + tid*R + j]
        cf2 win[R];                                         // win[r] = a[m + r - t]
#pragma unroll
        for (int r = 0; r < R; ++r) win[r] = ldc(base + r);
        int k = 0;
#ifdef MODEM_ABLATE_FIR
        k = K;
        acc[0][0] = win[0];
#endif
        for (; k + CH <= K; k += CH) {
            const float2* pc = base - (k + CH);   // positive ds_read immediates: pc[CH-1-c]
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                tx_mac<SPS, R>(acc, win, taps + (k + c) * SPS);
                shift_in<R>(win, ldc(pc + CH - 1 - c));
            }
        }
        for (; k < K; ++k) {
            tx_mac<SPS, R>(acc, win, taps + k * SPS);
            shift_in<R>(win, ldc(base - (k + 1)));
        }

        // 3. carrier mix + store straight from registers: R*SPS consecutive samples.
        const int64_t jt = m0 * SPS;                 // first sample of the tile (uniform)
        const int jl = tid * R * SPS;                // lane offset within the tile
        const int64_t jend = p.nsym * SPS;
#pragma unroll
        for (int i = 0; i < R * SPS; i += 2) {
            const int64_t j = jt + jl + i;
            if (j < jend) {
                const bool two = (i + 1 < R * SPS) && (j + 1 < jend);
                const cf2 a0 = acc[i / SPS][i % SPS];
                const int i1 = i + 1 < R * SPS ? i + 1 : i;
                const cf2 a1 = acc[i1 / SPS][i1 % SPS];
                tx_emit_off<OUT_MODE, OutT>(p, jt, jl + i, make_float2(a0.x, a0.y), make_float2(a1.x, a1.y), two);
            }
        }
        __syncthreads();   // the window is restaged next trip
    }
}

// ----------------------------------------------------------------------- TX on MFMA ----
// The zero-stuffed polyphase FIR as f32 matrix products (v_mfma_f32_16x16x4_f32 is an exact
// k-ordered fmaf chain, the same arithmetic as the VALU path, on the matrix pipe, leaving the
// VALU to the bit-exact carrier phase, sin/cos and mix):
//   rows i  = 16 row-blocks of SB = 16/SPS consecutive symbols,
//   cols j  = (symbol c in the block, phase p) -> sample SPS*c + p of the block (16 samples),
//   k  = o  = offset in a W = 4*NKS symbol window ending at the block's last symbol,
//   A[i][o] = a[block_i - PRE + o]  (complex: one chain for re, one for im; from LDS),
//   B[o][j] = h[p + SPS*(c + PRE - o)]  (banded tap matrix, constant: NKS VGPRs per lane).
// MAC efficiency = (SB + K - 1) / W (0.92 for 129 taps at sps 4). One wave computes one
// 16x16 output tile (256 samples) per 2*NKS MFMAs.
template <int SPS> struct TxMfmaCfg {
    static constexpr int SB = 16 / SPS;          // symbols per row-block
    static constexpr int NT = 256;               // 4 waves
    static constexpr int SUB = 4;                // 16x16 tiles per wave per tile
    static constexpr int TS = 4 * SUB * 16 * SB; // symbols per workgroup tile
};

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Keep a loaded value in its register: an opaque asm use stops the compiler from
// rematerialising the load inside the tile loop (where its vmcnt wait would also drain the
// next tile's prefetch, since vector-memory counters retire in issue order).
__device__ __forceinline__ void pin(float& v) { asm volatile("" : "+v"(v)); }

// acc_re/acc_im += sum_s A_s * B_s over NKS k-steps; A_s (complex) is read from LDS at
// arow[off(s)], PD k-steps ahead of its MFMA pair (explicit software pipeline: the
// scheduling barriers keep the compiler from collapsing it to one read of look-ahead).
template <int NKS, int PD, typename OffF>
__device__ __forceinline__ void mfma_chain(const float2* arow, OffF off, const float (&bf)[NKS],
                                           f32x4& dre, f32x4& dim) {
#ifdef MODEM_ABLATE_FIR
    const float2 a0 = arow[off(0)];
    dre[0] += a0.x * bf[0]; dim[0] += a0.y * bf[NKS - 1];
    return;
#endif
    float2 a[PD];
#pragma unroll
    for (int s = 0; s < PD && s < NKS; ++s) a[s] = arow[off(s)];
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
        const float2 cur = a[s % PD];
        if (s + PD < NKS) a[s % PD] = arow[off(s + PD)];
        dre = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.x, bf[s], dre, 0, 0, 0);
        dim = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.y, bf[s], dim, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// The same chain with B also read from LDS, at brow[4*s] (a Toeplitz band table: one
// conflict-free ds_read_b32 per k-step instead of NKS fragment registers per lane).
template <int NKS, int PD, typename OffF>
__device__ __forceinline__ void mfma_chain_lb(const float2* arow, OffF off, const float* brow,
                                              f32x4& dre, f32x4& dim) {
#ifdef MODEM_ABLATE_FIR
    const float2 a0 = arow[off(0)];
    dre[0] += a0.x * brow[0]; dim[0] += a0.y * brow[4];
    return;
#endif
    float2 a[PD];
    float b[PD];
#pragma unroll
    for (int s = 0; s < PD && s < NKS; ++s) {
        a[s] = arow[off(s)];
        b[s] = brow[4 * s];
    }
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
        const float2 cur = a[s % PD];
        const float cb = b[s % PD];
        if (s + PD < NKS) {
            a[s % PD] = arow[off(s + PD)];
            b[s % PD] = brow[4 * (s + PD)];
        }
        dre = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.x, cb, dre, 0, 0, 0);
        dim = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.y, cb, dim, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <int SPS, int NKS, int OUT_MODE, typename OutT>
struct TxMfma {
    using C = TxMfmaCfg<SPS>;
    static constexpr int SB = C::SB, NT = C::NT, SUB = C::SUB, TS = C::TS;
    static constexpr int PRE = 4 * NKS - SB;       // window symbols before a row-block
    static constexpr int NE = TS + PRE;            // symbols staged per tile
    static constexpr int U = (NE + NT - 1) / NT;   // prefetched staging slots per lane

    // Raw bits word of symbol m, BPS bytes (fast path: aligned, no leftover bits).
    template <int BPS>
    __device__ static uint64_t load_word(const uint8_t* bits, int64_t m) {
        const uint8_t* b = bits + m * BPS;
        if (BPS == 1) return *b;
        if (BPS == 2) return *reinterpret_cast<const uint16_t*>(b);
        if (BPS == 4) return *reinterpret_cast<const uint32_t*>(b);
        return *reinterpret_cast<const uint64_t*>(b);
    }

    // Slow staging: first tile (filter history), leftover bits, flush, any bps.
    __device__ static void stage_slow(const TxParams& p, float2* lds, const float2* lut_s, int64_t m0) {
        for (int e = threadIdx.x; e < NE; e += NT) {
            const int64_t m = m0 - PRE + e;
            lds[e] = m < 0 ? (m >= -(int64_t)(p.K - 1) ? p.hist[m + p.K - 1] : make_float2(0.f, 0.f))
                           : (m >= p.nsym_valid ? make_float2(0.f, 0.f) : lut_s[tx_symbol_index(p, m)]);
        }
    }

    // FIR of this wave's sub-tile q: D = sum_s A_s B_s (see the comment above TxMfmaCfg).
    __device__ static void fir(const float2* lds, int q, const float (&bf)[NKS], f32x4& dre, f32x4& dim) {
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        const int sb0 = (wave * SUB + q) * 16 * SB;
        const float2* arow = lds + sb0 + SB * (lane & 15) + (lane >> 4);
        dre = (f32x4){0.f, 0.f, 0.f, 0.f};
        dim = dre;
        mfma_chain<NKS, 4>(arow, [](int s) { return 4 * s; }, bf, dre, dim);
    }

    // Full 16x16 tile, carrier index < 2^32: four independent chains, unconditional stores.
    __device__ static void emit_full(const TxParams& p, int64_t jt, const f32x4& dre, const f32x4& dim) {
        const int lane = threadIdx.x & 63;
        const uint32_t nb = (uint32_t)(p.s0 + (uint64_t)jt);
        float zr[4], zi[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int off = 16 * (4 * (lane >> 4) + r) + (lane & 15);
            zr[r] = dre[r];
            zi[r] = dim[r];
#ifdef MODEM_ABLATE_MIX
            if (false) {
#else
            if (OUT_MODE != OUT_IQ_BASEBAND) {
#endif
                float sn, cs;
                sincos_phase(phase_from_f(p.w, (float)(nb + (uint32_t)off)), sn, cs);
                zr[r] = __builtin_fmaf(dre[r], cs, -(dim[r] * sn));
                zi[r] = __builtin_fmaf(dre[r], sn, dim[r] * cs);
            }
        }
#ifdef MODEM_ABLATE_STORE
#pragma unroll
        for (int r = 0; r < 4; ++r) asm volatile("" :: "v"(zr[r]), "v"(zi[r]));
#else
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t j = jt + 16 * (4 * (lane >> 4) + r) + (lane & 15);
            if (OUT_MODE == OUT_REAL) OutIO<OutT>::store_real_one(p.out, j, zr[r]);
            else OutIO<OutT>::store_one(p.out, j, zr[r], zi[r]);
        }
#endif
    }

    // Partial tile or carrier index >= 2^32: guarded, 64-bit indices.
    __device__ static void emit_edge(const TxParams& p, int64_t jt, const f32x4& dre, const f32x4& dim) {
        const int lane = threadIdx.x & 63;
        const int64_t jend = p.nsym * SPS;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int off = 16 * (4 * (lane >> 4) + r) + (lane & 15);
            if (jt + off < jend)
                tx_emit_off<OUT_MODE, OutT>(p, jt, off, make_float2(dre[r], dim[r]), make_float2(0.f, 0.f), false);
        }
    }

    // BPS > 0: bits aligned, no leftover bits, carrier index < 2^32 (the steady state).
    // BPS == 0: the general path (slow staging, guarded epilogue).
    template <int BPS>
    __device__ static void run(const TxParams& p, float2* lds, const float2* lut_s, const float (&bf)[NKS],
                               int64_t t0, int64_t t1) {
        const int tid = threadIdx.x;
        const int64_t nfull = p.nsym / TS;          // tiles with every sample inside the call
        const int64_t tf = BPS > 0 ? (t1 < nfull ? t1 : nfull) : t0;
        const int64_t mlast = p.nsym_valid - 1;
        auto inside = [&](int64_t m0) { return m0 - PRE >= 0 && m0 + TS <= p.nsym_valid; };
        uint64_t pre[U];
        // Always issued, address clamped into the call's bits: a fixed count of vector-memory
        // operations per trip keeps the compiler's vmcnt waits counted (never vmcnt(0)).
        auto prefetch = [&](int64_t m0) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                int64_t m = m0 - PRE + tid + NT * u;
                m = m < 0 ? 0 : (m > mlast ? mlast : m);
                pre[u] = load_word<BPS>(p.bits, m);
            }
        };
        if (BPS > 0 && t0 < tf && mlast >= 0) prefetch(t0 * TS);
        for (int64_t t = t0; t < tf; ++t) {
            const int64_t m0 = t * TS;
            if (inside(m0)) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int e = tid + NT * u;
                    if (e < NE) lds[e] = lut_s[word_index(pre[u], BPS)];
                }
            } else {
                stage_slow(p, lds, lut_s, m0);
            }
            __syncthreads();
            prefetch(m0 + TS);                       // next bits fly during the MFMAs
            // fully unrolled: a static store count lets the next trip wait vmcnt(#stores)
            // for its prefetched bits instead of draining this tile's stores
#pragma unroll
            for (int q = 0; q < SUB; ++q) {
                f32x4 dre, dim;
                fir(lds, q, bf, dre, dim);
                emit_full(p, (m0 + ((threadIdx.x >> 6) * SUB + q) * 16 * SB) * SPS, dre, dim);
            }
            __syncthreads();                         // the window is restaged next trip
        }
        for (int64_t t = tf > t0 ? tf : t0; t < t1; ++t) {   // partial / general tiles
            const int64_t m0 = t * TS;
            stage_slow(p, lds, lut_s, m0);
            __syncthreads();
#pragma unroll 1
            for (int q = 0; q < SUB; ++q) {
                f32x4 dre, dim;
                fir(lds, q, bf, dre, dim);
                emit_edge(p, (m0 + ((threadIdx.x >> 6) * SUB + q) * 16 * SB) * SPS, dre, dim);
            }
            __syncthreads();
        }
    }
};

template <int SPS, int NKS, int OUT_MODE, typename OutT>
__global__ __launch_bounds__(256) void tx_mfma(const TxParams p, const float* __restrict__ bfrag) {
    using K = TxMfma<SPS, NKS, OUT_MODE, OutT>;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2* lut_s = lds + ((K::NE + 1) & ~1);
    const int tid = threadIdx.x, lane = tid & 63;
    if (blockIdx.x == 0) tx_state_update(p);
    for (int i = tid; i < (1 << p.bps); i += K::NT) lut_s[i] = p.lut[i];
    float bf[NKS];                               // this lane's B fragments, one per k-step
#pragma unroll
    for (int s = 0; s < NKS; ++s) bf[s] = bfrag[s * 64 + lane];
#pragma unroll
    for (int s = 0; s < NKS; ++s) pin(bf[s]);
    __syncthreads();   // LUT visible
    const int64_t ntiles = (p.nsym + K::TS - 1) / K::TS;
    const int64_t t0 = ntiles * blockIdx.x / gridDim.x, t1 = ntiles * (blockIdx.x + 1) / gridDim.x;
    if (p.fast_bits && p.small_n) {              // one uniform switch: the tile loop is specialised
        switch (p.bps) {
        case 1: K::template run<1>(p, lds, lut_s, bf, t0, t1); return;
        case 2: K::template run<2>(p, lds, lut_s, bf, t0, t1); return;
        case 4: K::template run<4>(p, lds, lut_s, bf, t0, t1); return;
        case 8: K::template run<8>(p, lds, lut_s, bf, t0, t1); return;
        }
    }
    K::template run<0>(p, lds, lut_s, bf, t0, t1);
}

// Any samples-per-symbol: thread per output sample, symbols staged in LDS.
template <int OUT_MODE, typename OutT>
__global__ __launch_bounds__(256) void tx_generic(const TxParams p) {
    constexpr int NT = 256, TS = 64;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int K = p.K, SPS = p.sps;
    if (blockIdx.x == 0) tx_state_update(p);
    const int64_t m0 = (int64_t)blockIdx.x * TS;
    if (m0 >= p.nsym) return;
    for (int e = threadIdx.x; e < TS + K - 1; e += NT) lds[e] = tx_symbol_value(p, m0 - (K - 1) + e);
    __syncthreads();
    const int64_t nsym_here = p.nsym - m0 < TS ? p.nsym - m0 : TS;
    const int nsamp = (int)nsym_here * SPS;
    for (int i = threadIdx.x; i < nsamp; i += NT) {
        const int ml = i / SPS, q = i - ml * SPS;
        float yr = 0.f, yi = 0.f;
        for (int t = 0; t < K; ++t) {
            const float h = p.taps[t * SPS + q];
            const float2 a = lds[ml - t + K - 1];
            yr = __builtin_fmaf(a.x, h, yr);
            yi = __builtin_fmaf(a.y, h, yi);
        }
        tx_emit<OUT_MODE, OutT>(p, m0 * SPS + i, make_float2(yr, yi), make_float2(0.f, 0.f), false);
    }
}

// -------------------------------------------------------------------------------- RX ----
template <typename InT> struct InIO;
template <> struct InIO<float> {
    using Raw = float4;   // two consecutive samples
    __device__ static Raw load_raw(const void* x, int64_t q) {
        return *reinterpret_cast<const float4*>(reinterpret_cast<const float2*>(x) + q);
    }
    __device__ static void split(Raw v, float2& a, float2& b) {
        a = make_float2(v.x, v.y);
        b = make_float2(v.z, v.w);
    }
    __device__ static float2 load(const void* x, int64_t q) {
        return reinterpret_cast<const float2*>(x)[q];
    }
    __device__ static void load_pair(const void* x, int64_t q, float2& a, float2& b) {
        const float4 v = *reinterpret_cast<const float4*>(reinterpret_cast<const float2*>(x) + q);
        a = make_float2(v.x, v.y);
        b = make_float2(v.z, v.w);
    }
    __device__ static void copy(void* dst, int64_t i, const void* src, int64_t q) {
        reinterpret_cast<float2*>(dst)[i] = reinterpret_cast<const float2*>(src)[q];
    }
};
template <> struct InIO<__half> {
    using Raw = uint2;
    __device__ static Raw load_raw(const void* x, int64_t q) {
        return *reinterpret_cast<const uint2*>(reinterpret_cast<const __half2*>(x) + q);
    }
    __device__ static void split(Raw u, float2& a, float2& b) {
        a = __half22float2(*reinterpret_cast<const __half2*>(&u.x));
        b = __half22float2(*reinterpret_cast<const __half2*>(&u.y));
    }
    __device__ static float2 load(const void* x, int64_t q) {
        return __half22float2(reinterpret_cast<const __half2*>(x)[q]);
    }
    __device__ static void load_pair(const void* x, int64_t q, float2& a, float2& b) {
        const uint2 u = *reinterpret_cast<const uint2*>(reinterpret_cast<const __half2*>(x) + q);
        a = __half22float2(*reinterpret_cast<const __half2*>(&u.x));
        b = __half22float2(*reinterpret_cast<const __half2*>(&u.y));
    }
    __device__ static void copy(void* dst, int64_t i, const void* src, int64_t q) {
        reinterpret_cast<__half2*>(dst)[i] = reinterpret_cast<const __half2*>(src)[q];
    }
};

enum { MIX_COMPLEX = 0, MIX_REFERENCE_REAL = 1 };
enum { SLICER_NONE = 0, SLICER_NEAREST = 1, SLICER_QAM_AXIS = 2 };

// Sample q of the chunk (q < 0: history; q >= N: past the chunk, zero).
template <typename InT>
__device__ __forceinline__ float2 rx_sample(const RxParams& p, int64_t q) {
    if (q < -(int64_t)p.HL) return make_float2(0.f, 0.f);
    if (q >= 0) return q < p.N ? InIO<InT>::load(p.x, q) : make_float2(0.f, 0.f);
    return InIO<InT>::load(p.hist, q + p.HL);
}

template <typename InT>
__device__ __forceinline__ void rx_pair(const RxParams& p, int64_t q, float2& a, float2& b) {
    if (q >= 0 && q + 1 < p.N && p.x_aligned16) {
        InIO<InT>::load_pair(p.x, q, a, b);
    } else {
        a = rx_sample<InT>(p, q);
        b = rx_sample<InT>(p, q + 1);
    }
}

// x * e^{-j phase} (or the reference's x.re * (cos, -sin), demodulator.rs:46,53-54) for
// stream index n = nb + off (nb wave-uniform).
template <int MIX>
__device__ __forceinline__ float2 rx_mix(const RxParams& p, int64_t nb, int off, float2 x) {
    if (nb + off < 0) return make_float2(0.f, 0.f);   // before the stream: zero history
    float s, c;
    sincos_phase(carrier_phase_off(p.w, p.c0 + (uint64_t)nb, off, p.small_n), s, c);
    if (MIX == MIX_REFERENCE_REAL) return make_float2(x.x * c, x.x * -s);
    return make_float2(__builtin_fmaf(x.y, s, x.x * c), __builtin_fmaf(-x.x, s, x.y * c));
}

__device__ __forceinline__ uint8_t rx_slice(const RxParams& p, float re, float im) {
#pragma clang fp contract(off)
    if (p.slicer_kind == SLICER_QAM_AXIS) {
        const int ms = (int)p.max_symbol;
        const float fi = (re * p.inv_scale + p.max_symbol) * 0.5f;
        const float fq = (im * p.inv_scale + p.max_symbol) * 0.5f;
        const int si = (int)__builtin_fminf(__builtin_fmaxf(__builtin_rintf(fi), 0.f), (float)ms);
        const int sq = (int)__builtin_fminf(__builtin_fmaxf(__builtin_rintf(fq), 0.f), (float)ms);
        return (uint8_t)((si << p.bits_per_carrier) | sq);
    }
    cfloat* lut = (cfloat*)p.slut;
    const int n = 1 << p.bps;
    uint32_t best = 0;
    float bd = __builtin_inff();
    for (int k = 0; k < n; ++k) {
        const float dr = re - lut[2 * k], di = im - lut[2 * k + 1];
        const float d = dr * dr + di * di;
        if (d < bd) { bd = d; best = (uint32_t)k; }
    }
    return (uint8_t)best;
}

template <typename OutT>
__device__ __forceinline__ void rx_emit(const RxParams& p, int64_t o, float re, float im) {
#ifdef MODEM_ABLATE_STORE
    asm volatile("" :: "v"(re), "v"(im));
    return;
#endif
    if (p.out_iq) OutIO<OutT>::store_one(p.out_iq, o, re, im);
    if (p.out_sym && p.slicer_kind != SLICER_NONE) p.out_sym[o] = rx_slice(p, re, im);
}

template <typename InT>
__device__ void rx_state_update(const RxParams& p) {
    for (int i = threadIdx.x; i < p.HL; i += blockDim.x) {
        const int64_t q = p.N - p.HL + i;
        if (q >= 0) InIO<InT>::copy(p.hist_new, i, p.x, q);
        else InIO<InT>::copy(p.hist_new, i, p.hist, q + p.HL);
    }
}

template <int DEC> struct RxCfg {
    static constexpr int R = DEC == 1 ? 9 : DEC == 2 ? 7 : DEC == 4 ? 5 : DEC == 8 ? 3 : 1;  // odd
    static constexpr int NT = 256;
    static constexpr int TS = NT * R;   // output symbols per tile
    static constexpr int CH = 8;
    // taps per branch the prefetch ring covers (longer filters take the slow staging path)
    static constexpr int KMAX = DEC == 1 ? 65 : DEC == 8 ? 65 : 33;
    // sample pairs prefetched per lane: covers (TS + KMAX - 1) * DEC samples plus one
    // (a tile whose first sample is odd starts its pairs one sample early)
    static constexpr int U = ((TS + KMAX - 1) * DEC + 1 + 2 * NT - 1) / (2 * NT);
};

template <int R>
__device__ __forceinline__ void rx_mac(cf2 (&acc)[R], const cf2 (&win)[R], float h) {
#pragma unroll
    for (int i = 0; i < R; ++i) acc[i] = cmac(win[i], h, acc[i]);
}

// Plane stride (float2 elements): TS + K rounded to an odd count (bank spread of the
// per-plane base); lanes read with stride R (odd) -> conflict-free ds_read_b64.
__host__ __device__ inline int rx_plane_stride(int TS, int K) { return (TS + K) | 1; }

// Rare path (first / last tile of a chunk, unaligned input, carrier index >= 2^32): one
// sample at a time with full 64-bit bookkeeping, as one rolled loop under a uniform branch
// (never called out of line: a call would push the kernel arguments to per-lane scratch).
template <int DEC, typename InT, int MIX>
__device__ __forceinline__ void rx_stage_slow(const RxParams& p, float2* lds, int PS, int NS,
                                           int64_t q_lo) {
    const int64_t n_lo = q_lo + p.n_start;
    for (int e = threadIdx.x; e < NS; e += blockDim.x) {
        const float2 z = rx_mix<MIX>(p, n_lo, e, rx_sample<InT>(p, q_lo + e));
        const int em = e / DEC, b = DEC - 1 - (e - em * DEC);   // z_b[m] = z[m*DEC + D - b]
        lds[b * PS + 1 + em] = z;
    }
}

// Steady state: every staged sample lies inside the chunk and below carrier index 2^32.
// Slot u of lane tid holds samples e = 2*(tid + NT*u) - PAR + {0,1}; the per-slot part of
// every index is a compile-time constant (NT*2/DEC plane elements per slot), so the LDS
// stores use immediate offsets and the phase needs one 32-bit add.
template <int DEC, typename InT, int MIX, int PAR, int U, int NT>
__device__ __forceinline__ void rx_stage_fast(const RxParams& p, float2* lds, int PS, int NS,
                                              uint32_t nb32, const typename InIO<InT>::Raw (&pre)[U]) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        float2 x[2];
        InIO<InT>::split(pre[u], x[0], x[1]);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int el = 2 * tid - PAR + j;           // lane part of e (>= -1)
            const int e = el + 2 * NT * u;
            if (e >= 0 && e < NS) {
                float s, c;
#ifdef MODEM_ABLATE_MIX
                s = 0.f; c = (float)(nb32 + (uint32_t)e);
#else
                sincos_phase(phase_from_f(p.w, (float)(nb32 + (uint32_t)e)), s, c);
#endif
                float2 z;
                if (MIX == MIX_REFERENCE_REAL) z = make_float2(x[j].x * c, x[j].x * -s);
                else z = make_float2(__builtin_fmaf(x[j].y, s, x[j].x * c),
                                     __builtin_fmaf(-x[j].x, s, x[j].y * c));
                const int em_l = (el + DEC) / DEC - 1;  // floor(el / DEC), el >= -1
                const int b = DEC - 1 - (el + DEC - (em_l + 1) * DEC);
                lds[b * PS + 1 + em_l + (2 * NT / DEC) * u] = z;
            }
        }
    }
}

template <int DEC, typename InT, int MIX, typename OutT>
__global__ __launch_bounds__(256) void rx_fast(const RxParams p) {
    using C = RxCfg<DEC>;
    using IO = InIO<InT>;
    using Raw = typename IO::Raw;
    constexpr int R = C::R, NT = C::NT, TS = C::TS, CH = C::CH, U = C::U;
    static_assert((2 * NT) % DEC == 0, "slot stride must be whole plane elements");
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int tid = threadIdx.x;
    const int K = p.K;
    const int PS = rx_plane_stride(TS, K);
    const int NS = (TS + K - 1) * DEC;             // samples staged per tile
    if (blockIdx.x == 0) rx_state_update<InT>(p);

    // Persistent workgroup: a balanced contiguous range of tiles of kept instants.
    const int64_t ntiles = (p.nout + TS - 1) / TS;
    const int64_t t0 = ntiles * blockIdx.x / gridDim.x, t1 = ntiles * (blockIdx.x + 1) / gridDim.x;
    // tile t stages stream samples n_lo(t) .. n_lo(t) + NS - 1; chunk index q = n - n_start
    auto q_lo_of = [&](int64_t t) {
        return (p.k_first + t * TS) * DEC + p.D - (int64_t)K * DEC + 1 - p.n_start;
    };
    // A tile is "inside" when its prefetched slots are whole pairs of this chunk.
    const bool pf = p.x_aligned16 && p.small_n && NS + 1 <= 2 * NT * U;   // workgroup-uniform
    auto inside = [&](int64_t q_lo) {
        const int64_t qb = q_lo - (q_lo & 1);
        return pf && qb >= 0 && qb + 2 * NT * U <= p.N;
    };
    Raw pre[U];
    auto prefetch = [&](int64_t q_lo) {
        const Raw* xb = reinterpret_cast<const Raw*>(p.x) + ((q_lo - (q_lo & 1)) >> 1);
#pragma unroll
        for (int u = 0; u < U; ++u) pre[u] = xb[tid + NT * u];
    };
    if (t0 < t1 && inside(q_lo_of(t0))) prefetch(q_lo_of(t0));

    cfloat* taps = (cfloat*)p.taps;
    for (int64_t t = t0; t < t1; ++t) {
        const int64_t q_lo = q_lo_of(t);
        // 1. mix the tile's samples into DEC polyphase planes.
        if (inside(q_lo)) {
            const uint32_t nb32 = (uint32_t)(p.c0 + (uint64_t)(q_lo - (q_lo & 1) + p.n_start));
            if (q_lo & 1) rx_stage_fast<DEC, InT, MIX, 1, U, NT>(p, lds, PS, NS, nb32 + 1u, pre);
            else rx_stage_fast<DEC, InT, MIX, 0, U, NT>(p, lds, PS, NS, nb32, pre);
        } else {
            rx_stage_slow<DEC, InT, MIX>(p, lds, PS, NS, q_lo);
        }
        __syncthreads();
        if (t + 1 < t1) {                       // next tile's samples fly during the filter
            const int64_t qn = q_lo_of(t + 1);
            if (inside(qn)) prefetch(qn);
        }


        // 2. matched filter at the kept instants, R consecutive outputs per lane.
        cf2 acc[R];
#pragma unroll
        for (int i = 0; i < R; ++i) acc[i] = (cf2){0.f, 0.f};
#pragma unroll 1
        for (int b = 0; b < DEC; ++b) {
            const float2* base = lds + b * PS + 1 + tid * R + (K - 1);   // base[j] = z_b[k+j]
            cfloat* hb = taps + b * K;
            cf2 win[R];
#pragma unroll
            for (int i = 0; i < R; ++i) win[i] = ldc(base + i);
            int k = 0;
#ifdef MODEM_ABLATE_FIR
            k = K;
            acc[0] += win[0];
#endif
            for (; k + CH <= K; k += CH) {
                const float2* pc = base - (k + CH);   // positive ds_read immediates
#pragma unroll
                for (int c = 0; c < CH; ++c) {
                    rx_mac<R>(acc, win, hb[k + c]);
                    shift_in<R>(win, ldc(pc + CH - 1 - c));
                }
            }
            for (; k < K; ++k) {
                rx_mac<R>(acc, win, hb[k]);
                shift_in<R>(win, ldc(base - (k + 1)));
            }
        }

        // 3. decisions + stores.
        const float g = MIX == MIX_REFERENCE_REAL ? 2.0f : 1.0f;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int64_t o = t * TS + tid * R + i;
            if (o < p.nout) rx_emit<OutT>(p, o, g * acc[i].x, g * acc[i].y);
        }
        __syncthreads();   // planes are restaged next trip
    }
}

// ----------------------------------------------------------------------- RX on MFMA ----
// Matched filter at the kept instants as f32 matrix products (v_mfma_f32_16x16x4_f32):
//   rows i = 16 groups of 16 consecutive kept instants, cols c = instant in the group,
//   k = w  = offset in a W = 4*NKS sample window ending at the group's last instant,
//   A[i][w] = z[start_i + w]  (mixed input from LDS; one chain for re, one for im),
//   B[w][c] = h[W - 1 - w - (15 - c)*DEC]  (banded tap matrix: NKS VGPRs per lane).
// MAC efficiency = L / W (0.67 for 129 taps at decimation 4). One wave: one 16x16 tile
// (256 instants) per 2*NKS MFMAs. LDS keeps the mixed samples in natural order with 2 pad
// samples after every RW = 16*DEC (one row of A), so the 16 rows of a read land in distinct
// banks and every k-step is a compile-time immediate offset.
template <int DEC> struct RxMfmaCfg {
    static constexpr int NT = 256;               // 4 waves
    static constexpr int TS = 4 * 256;           // kept instants per workgroup tile
    static constexpr int RW = 16 * DEC;          // samples per A row
};
__host__ __device__ constexpr int rxm_pos(int e, int RW) { return e + 2 * (e / RW); }

// What the steady-state epilogue writes: baseband IQ, QAM-axis decisions, or both
// (RXE_GEN: any other combination, guarded per store).
enum { RXE_GEN = 0, RXE_IQ = 1, RXE_SYM = 2, RXE_IQSYM = 3 };

__device__ __forceinline__ uint8_t rx_slice_qam(const RxParams& p, float re, float im) {
#pragma clang fp contract(off)
    const int ms = (int)p.max_symbol;
    const float fi = (re * p.inv_scale + p.max_symbol) * 0.5f;
    const float fq = (im * p.inv_scale + p.max_symbol) * 0.5f;
    // clamp before the conversion: huge / NaN inputs stay defined (fmax drops a NaN)
    const int si = (int)__builtin_fminf(__builtin_fmaxf(__builtin_rintf(fi), 0.f), (float)ms);
    const int sq = (int)__builtin_fminf(__builtin_fmaxf(__builtin_rintf(fq), 0.f), (float)ms);
    return (uint8_t)((si << p.bits_per_carrier) | sq);
}

template <int DEC, int NKS, typename InT, int MIX, typename OutT>
struct RxMfma {
    using C = RxMfmaCfg<DEC>;
    using IO = InIO<InT>;
    using Raw = typename IO::Raw;
    static constexpr int NT = C::NT, TS = C::TS, RW = C::RW;
    static constexpr int W = 4 * NKS;
    static constexpr int NS = (TS - 16) * DEC + W;            // samples staged per tile
    static constexpr int U = (NS + 1 + 2 * NT - 1) / (2 * NT); // prefetched sample pairs per lane
    static constexpr float GAIN = MIX == MIX_REFERENCE_REAL ? 2.0f : 1.0f;

    // Tile t stages chunk samples q_lo .. q_lo + NS - 1 (window start of its first row).
    __device__ static int64_t q_lo_of(const RxParams& p, int64_t t) {
        return (p.k_first + t * TS) * DEC + p.D + 15 * DEC - W + 1 - p.n_start;
    }

    // Steady state: the tile's samples are whole pairs of this chunk, carrier index < 2^32,
    // every instant is kept. PAR = q_lo & 1 is the same for every tile of a call (TS*DEC even).
    template <int PAR>
    __device__ static void stage_fast(const RxParams& p, float2* lds, uint32_t nb32, const Raw (&pre)[U]) {
        const int tid = threadIdx.x;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float2 x[2];
            IO::split(pre[u], x[0], x[1]);
            const int e0 = 2 * (tid + NT * u) - PAR;     // stage index of x[0]
            float2 z[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                float sn, cs;
#ifdef MODEM_ABLATE_MIX
                sn = 0.f; cs = (float)(nb32 + (uint32_t)(2 * (tid + NT * u) + j));
#else
                sincos_phase(phase_from_f(p.w, (float)(nb32 + (uint32_t)(2 * (tid + NT * u) + j))), sn, cs);
#endif
                if (MIX == MIX_REFERENCE_REAL) z[j] = make_float2(x[j].x * cs, x[j].x * -sn);
                else z[j] = make_float2(__builtin_fmaf(x[j].y, sn, x[j].x * cs),
                                        __builtin_fmaf(-x[j].x, sn, x[j].y * cs));
            }
            // Only the first and last slots can fall outside [0, NS): the other guards are
            // compile-time true, so the slots' chains interleave without branches.
            const bool last = (u + 1) * 2 * NT > NS - 1;
            if (PAR == 0) {
                if (!last || e0 < NS)   // a pair never straddles a padded row (RW even): one 16-B store
                    *reinterpret_cast<float4*>(lds + rxm_pos(e0, RW)) = make_float4(z[0].x, z[0].y, z[1].x, z[1].y);
            } else {
                if ((u > 0 || e0 >= 0) && (!last || e0 < NS)) lds[rxm_pos(e0, RW)] = z[0];
                if (!last || e0 + 1 < NS) lds[rxm_pos(e0 + 1, RW)] = z[1];
            }
        }
    }

    // First / last tiles of a chunk, unaligned input, carrier index >= 2^32: per sample.
    __device__ static void stage_slow(const RxParams& p, float2* lds, int64_t q_lo) {
        const int64_t n_lo = q_lo + p.n_start;
        for (int e = threadIdx.x; e < NS; e += NT)
            lds[rxm_pos(e, RW)] = rx_mix<MIX>(p, n_lo, e, rx_sample<InT>(p, q_lo + e));
    }

    static constexpr int TBL = rx_mfma_table_len(DEC, NKS);   // band table floats
    static constexpr int LDS_SAMPLES = rxm_pos(NS, RW) + 2;      // float2 slots before the table

    // One 16x16 tile per wave: instants kt + 16*i + c. Lane (g, c) reads A from row c of its
    // wave's block and B[4s + g][c] = T[4s + g + (15 - c)*DEC] from the band table.
    __device__ static void fir(const float2* lds, const float* tbl, f32x4& dre, f32x4& dim) {
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        const float2* arow = lds + rxm_pos(wave * 16 * RW, RW) + (lane & 15) * (RW + 2) + (lane >> 4);
        const float* brow = tbl + (lane >> 4) + (15 - (lane & 15)) * DEC;
        dre = (f32x4){0.f, 0.f, 0.f, 0.f};
        dim = dre;
        mfma_chain_lb<NKS, 4>(arow, [](int s) { return 4 * s + 2 * ((4 * s) / RW); }, brow, dre, dim);
    }

    // D[row][col]: row = 4*(lane>>4) + r, col = lane&15 -> instant ot + 16*row + col.
    template <int EM>
    __device__ static void emit_full(const RxParams& p, int64_t ot, const f32x4& dre, const f32x4& dim) {
        const int lane = threadIdx.x & 63;
#ifdef MODEM_ABLATE_STORE
#pragma unroll
        for (int r = 0; r < 4; ++r) asm volatile("" :: "v"(dre[r]), "v"(dim[r]));
        return;
#endif
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int off = 16 * (4 * (lane >> 4) + r) + (lane & 15);
            const float re = GAIN * dre[r], im = GAIN * dim[r];
            if (EM == RXE_GEN) {
                rx_emit<OutT>(p, ot + off, re, im);
                continue;
            }
            if (EM & RXE_IQ) OutIO<OutT>::store_one(p.out_iq, ot + off, re, im);
            if (EM & RXE_SYM) p.out_sym[ot + off] = rx_slice_qam(p, re, im);
        }
    }

    __device__ static void emit_edge(const RxParams& p, int64_t ot, const f32x4& dre, const f32x4& dim) {
        const int lane = threadIdx.x & 63;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t o = ot + 16 * (4 * (lane >> 4) + r) + (lane & 15);
            if (o < p.nout) rx_emit<OutT>(p, o, GAIN * dre[r], GAIN * dim[r]);
        }
    }

    // Tiles of [t0, t1). When the call's input is 16-B aligned and its carrier indices stay
    // below 2^32, the run of "full" tiles (all staged samples inside the chunk, all 1024
    // instants kept) goes through the prefetched loop, whose epilogue EM stores unconditionally;
    // the first and last tiles of the chunk take the general path. PAR = q_lo & 1 is the same
    // for every tile of a call (TS*DEC is even).
    template <int EM>
    __device__ static void run(const RxParams& p, float2* lds, const float* bf, int64_t t0, int64_t t1) {
        const int tid = threadIdx.x, wave = tid >> 6;
        const int64_t npairs = p.N >> 1;
        const bool fast = p.x_aligned16 && p.small_n;
        const int PAR = (int)(q_lo_of(p, 0) & 1);
        auto full = [&](int64_t t) {
            const int64_t qb = q_lo_of(p, t) - PAR;
            return fast && qb >= 0 && qb + 2 * NT * U <= p.N && (t + 1) * TS <= p.nout;
        };
        Raw pre[U];
        // Always issued, base clamped into the chunk: a fixed count of vector-memory operations
        // per trip keeps the compiler's vmcnt waits counted (a non-full next tile is restaged).
        auto prefetch = [&](int64_t t) {
            int64_t base = (q_lo_of(p, t) - PAR) >> 1;
            base = base > npairs - NT * U ? npairs - NT * U : base;
            const Raw* xb = reinterpret_cast<const Raw*>(p.x) + base;
#pragma unroll
            for (int u = 0; u < U; ++u) pre[u] = xb[tid + NT * u];
        };
        int64_t t = t0;
        while (t < t1) {
            if (full(t)) {
                prefetch(t);
                for (; t < t1 && full(t); ++t) {
                    const int64_t n_lo = q_lo_of(p, t) + p.n_start;
                    const uint32_t nb32 = (uint32_t)(p.c0 + (uint64_t)(n_lo - PAR));
                    if (PAR) stage_fast<1>(p, lds, nb32, pre);   // uniform; no memory-counter ops inside
                    else stage_fast<0>(p, lds, nb32, pre);
                    __syncthreads();
                    prefetch(t + 1);                       // next samples fly during the MFMAs
                    f32x4 dre, dim;
                    fir(lds, bf, dre, dim);
                    emit_full<EM>(p, t * TS + wave * 256, dre, dim);
                    __syncthreads();                       // LDS is restaged next trip
                }
            } else {
                stage_slow(p, lds, q_lo_of(p, t));
                __syncthreads();
                f32x4 dre, dim;
                fir(lds, bf, dre, dim);
                emit_edge(p, t * TS + wave * 256, dre, dim);
                __syncthreads();
                ++t;
            }
        }
    }
};

template <int DEC, int NKS, typename InT, int MIX, typename OutT>
__global__ __launch_bounds__(256) void rx_mfma(const RxParams p, const float* __restrict__ bfrag) {
    using K = RxMfma<DEC, NKS, InT, MIX, OutT>;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    if (blockIdx.x == 0) rx_state_update<InT>(p);
    float* bf = reinterpret_cast<float*>(lds + K::LDS_SAMPLES);   // band table, read-only below
    for (int j = threadIdx.x; j < K::TBL; j += K::NT) bf[j] = bfrag[j];
    __syncthreads();
    const int64_t ntiles = (p.nout + K::TS - 1) / K::TS;
    const int64_t t0 = ntiles * blockIdx.x / gridDim.x, t1 = ntiles * (blockIdx.x + 1) / gridDim.x;
    if (t0 >= t1) return;
    // f32 input with the complex mix (the loopback chain): the epilogue is specialised on what
    // it stores, so the tile loop's store count is static. Other variants share the guarded one.
    if (std::is_same<InT, float>::value && MIX == MIX_COMPLEX) {
        const bool qam = p.slicer_kind == SLICER_QAM_AXIS && p.out_sym;
        if (p.out_iq && qam) { K::template run<RXE_IQSYM>(p, lds, bf, t0, t1); return; }
        if (p.out_iq && !p.out_sym) { K::template run<RXE_IQ>(p, lds, bf, t0, t1); return; }
        if (!p.out_iq && qam) { K::template run<RXE_SYM>(p, lds, bf, t0, t1); return; }
    }
    K::template run<RXE_GEN>(p, lds, bf, t0, t1);
}

// Any decimation: thread per kept instant, mixed samples staged in natural order.
template <typename InT, int MIX, typename OutT>
__global__ __launch_bounds__(64) void rx_generic(const RxParams p) {
    constexpr int TS = 64;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int L = p.L, DEC = p.decim;
    if (blockIdx.x == 0) rx_state_update<InT>(p);
    const int64_t k0 = p.k_first + (int64_t)blockIdx.x * TS;
    if ((int64_t)blockIdx.x * TS >= p.nout) return;
    const int64_t n_lo = k0 * DEC + p.D - (L - 1);
    const int NS = (TS - 1) * DEC + L;
    for (int e = threadIdx.x; e < NS; e += TS)
        lds[e] = rx_mix<MIX>(p, n_lo, e, rx_sample<InT>(p, n_lo + e - p.n_start));
    __syncthreads();
    const int64_t o = (int64_t)blockIdx.x * TS + threadIdx.x;
    if (o >= p.nout) return;
    const int c = threadIdx.x * DEC + L - 1;
    float yr = 0.f, yi = 0.f;
    for (int j = 0; j < L; ++j) {
        const float h = p.taps[(j % DEC) * p.K + j / DEC];
        yr = __builtin_fmaf(lds[c - j].x, h, yr);
        yi = __builtin_fmaf(lds[c - j].y, h, yi);
    }
    const float g = MIX == MIX_REFERENCE_REAL ? 2.0f : 1.0f;
    rx_emit<OutT>(p, o, g * yr, g * yi);
}

// ------------------------------------------------------------------- FIRFilter (real) ----
// y[n] = sum_{k<L} h[k] x[n-k] (fir.rs:18-34); 256 lanes x 16 outputs per workgroup.
constexpr int kFirR = 16, kFirNT = 256, kFirTS = kFirR * kFirNT;

__global__ __launch_bounds__(256) void fir_real(const FirParams p) {
    extern __shared__ __attribute__((aligned(16))) float flds[];
    const int tid = threadIdx.x, L = p.L;
    if (blockIdx.x == 0)
        for (int i = tid; i < L - 1; i += kFirNT) {
            const int64_t q = p.N - (L - 1) + i;
            p.hist_new[i] = q >= 0 ? p.x[q] : p.hist[q + L - 1];
        }
    const int64_t n0 = (int64_t)blockIdx.x * kFirTS;
    if (n0 >= p.N) return;
    for (int e = tid; e < kFirTS + L - 1; e += kFirNT) {
        const int64_t q = n0 - (L - 1) + e;
        flds[1 + e] = q < 0 ? p.hist[q + L - 1] : (q < p.N ? p.x[q] : 0.f);
    }
    __syncthreads();
    float acc[kFirR];
#pragma unroll
    for (int r = 0; r < kFirR; ++r) acc[r] = 0.f;
    const float* base = flds + 1 + tid * kFirR + (L - 1);
    float win[kFirR];
#pragma unroll
    for (int r = 0; r < kFirR; ++r) win[r] = base[r];
    cfloat* taps = (cfloat*)p.taps;
    int k = 0;
    for (; k + 8 <= L; k += 8) {
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const float h = taps[k + c];
#pragma unroll
            for (int r = 0; r < kFirR; ++r) acc[r] = __builtin_fmaf(win[r], h, acc[r]);
#pragma unroll
            for (int r = kFirR - 1; r > 0; --r) win[r] = win[r - 1];
            win[0] = base[-(k + c + 1)];
        }
    }
    for (; k < L; ++k) {
        const float h = taps[k];
#pragma unroll
        for (int r = 0; r < kFirR; ++r) acc[r] = __builtin_fmaf(win[r], h, acc[r]);
#pragma unroll
        for (int r = kFirR - 1; r > 0; --r) win[r] = win[r - 1];
        win[0] = base[-(k + 1)];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kFirR; ++r) flds[tid * kFirR + r] = acc[r];
    __syncthreads();
    const int64_t nh = p.N - n0 < kFirTS ? p.N - n0 : kFirTS;
    for (int i = tid; i < nh; i += kFirNT) p.y[n0 + i] = flds[i];
}

// ----------------------------------------------------------- carrier phases (tests) ----
__global__ __launch_bounds__(256) void carrier_phases(float w, uint64_t s0, size_t n, int small_n,
                                                      float* out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = carrier_phase(w, s0 + i, small_n != 0);
}

hipError_t launch_phases(float w, uint64_t s0, size_t n, float* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const int small_n = (s0 + n) <= (1ull << 32) ? 1 : 0;
    hipLaunchKernelGGL(carrier_phases, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, w, s0, n,
                       small_n, out);
    return hipGetLastError();
}

// ------------------------------------------------------------------- splitmix64 bits ----
__global__ __launch_bounds__(256) void prng_bits(uint64_t seed, uint8_t* out, size_t nbits) {
    const size_t w = (size_t)blockIdx.x * blockDim.x + threadIdx.x;   // one 64-bit word
    if (w * 64 >= nbits) return;
    uint64_t z = seed + (uint64_t)(w + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z = z ^ (z >> 31);
    const size_t b0 = w * 64;
    if (b0 + 64 <= nbits && (reinterpret_cast<uintptr_t>(out + b0) & 15) == 0) {
        uint4* o = reinterpret_cast<uint4*>(out + b0);
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            uint32_t wd[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int bit = v * 16 + k * 4;
                wd[k] = (uint32_t)((z >> bit) & 1) | (uint32_t)((z >> (bit + 1)) & 1) << 8 |
                        (uint32_t)((z >> (bit + 2)) & 1) << 16 | (uint32_t)((z >> (bit + 3)) & 1) << 24;
            }
            o[v] = make_uint4(wd[0], wd[1], wd[2], wd[3]);
        }
    } else {
        for (size_t i = b0; i < nbits; ++i) out[i] = (uint8_t)((z >> (i - b0)) & 1);
    }
}

// ---------------------------------------------------------------------- dispatch ----
// Persistent grids: resident workgroups per CU (occupancy API, cached per kernel and LDS
// size) x CUs, never more than the number of tiles.
static int device_cus() {
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (cus[dev] == 0) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cus[dev] = n;
    }
    return cus[dev];
}

static std::mutex g_occ_mu;
static std::map<std::pair<const void*, size_t>, int> g_occ;

static int resident_blocks(const void* kernel, int threads, size_t lds) {
    std::lock_guard<std::mutex> lk(g_occ_mu);
    auto key = std::make_pair(kernel, lds);
    auto it = g_occ.find(key);
    if (it != g_occ.end()) return it->second;
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, threads, lds) != hipSuccess || occ <= 0) {
        (void)hipGetLastError();
        occ = 1;
    }
    g_occ[key] = occ;
    return occ;
}

static unsigned persistent_grid(const void* kernel, int threads, size_t lds, int64_t ntiles) {
    const int64_t cap = (int64_t)resident_blocks(kernel, threads, lds) * device_cus();
    const int64_t g = ntiles < cap ? ntiles : cap;
    return (unsigned)(g > 0 ? g : 1);
}

template <int SPS, int OM, typename OutT>
static hipError_t tx_go(const TxParams& p, hipStream_t s) {
    using C = TxCfg<SPS>;
    const int64_t ntiles = (p.nsym + C::TS - 1) / C::TS;
    const size_t lds = ((size_t)((C::TS + p.K + 2) & ~1) + ((size_t)1 << p.bps)) * sizeof(float2);
    const void* k = reinterpret_cast<const void*>(&tx_fast<SPS, OM, OutT>);
    hipLaunchKernelGGL((tx_fast<SPS, OM, OutT>), dim3(persistent_grid(k, C::NT, lds, ntiles)),
                       dim3(C::NT), lds, s, p);
    return hipGetLastError();
}

template <int OM, typename OutT>
static hipError_t tx_sps(const TxParams& p, int sps, hipStream_t s) {
    switch (sps) {
    case 1: return tx_go<1, OM, OutT>(p, s);
    case 2: return tx_go<2, OM, OutT>(p, s);
    case 4: return tx_go<4, OM, OutT>(p, s);
    case 8: return tx_go<8, OM, OutT>(p, s);
    case 16: return tx_go<16, OM, OutT>(p, s);
    default: {
        const int64_t nblk = (p.nsym + 63) / 64;
        const size_t lds = (size_t)(64 + p.K) * sizeof(float2);
        hipLaunchKernelGGL((tx_generic<OM, OutT>), dim3((unsigned)(nblk > 0 ? nblk : 1)), dim3(256),
                           lds, s, p);
        return hipGetLastError();
    }
    }
}

template <typename OutT>
static hipError_t tx_mode(const TxParams& p, int sps, int out_mode, hipStream_t s) {
    switch (out_mode) {
    case OUT_IQ_MIXED: return tx_sps<OUT_IQ_MIXED, OutT>(p, sps, s);
    case OUT_IQ_BASEBAND: return tx_sps<OUT_IQ_BASEBAND, OutT>(p, sps, s);
    default: return tx_sps<OUT_REAL, OutT>(p, sps, s);
    }
}

template <int SPS, int NKS, int OM, typename OutT>
static hipError_t txm_go(const TxParams& p, const float* bfrag, hipStream_t s) {
    using C = TxMfmaCfg<SPS>;
    constexpr int NE = TxMfma<SPS, NKS, OM, OutT>::NE;
    const int64_t ntiles = (p.nsym + C::TS - 1) / C::TS;
    const size_t lds = ((size_t)((NE + 1) & ~1) + ((size_t)1 << p.bps)) * sizeof(float2);
    const void* k = reinterpret_cast<const void*>(&tx_mfma<SPS, NKS, OM, OutT>);
    hipLaunchKernelGGL((tx_mfma<SPS, NKS, OM, OutT>), dim3(persistent_grid(k, C::NT, lds, ntiles)),
                       dim3(C::NT), lds, s, p, bfrag);
    return hipGetLastError();
}

template <int OM, typename OutT>
static hipError_t txm_sel(const TxParams& p, int sps, int nks, const float* bfrag, hipStream_t s) {
#define TXM(S, N) if (sps == S && nks == N) return txm_go<S, N, OM, OutT>(p, bfrag, s);
    TXM(4, 3) TXM(4, 5) TXM(4, 9) TXM(4, 17) TXM(4, 33)
    TXM(8, 5) TXM(8, 9) TXM(8, 17) TXM(8, 33)
    TXM(2, 5) TXM(2, 9) TXM(2, 17)
    TXM(16, 3) TXM(16, 5) TXM(16, 9) TXM(16, 17)
#undef TXM
    return hipErrorInvalidValue;
}

int tx_mfma_ksteps(int sps, int K) {
    if (sps != 2 && sps != 4 && sps != 8 && sps != 16) return 0;
    const int need = (16 / sps + K - 1 + 3) / 4;
    static const int steps[] = {3, 5, 9, 17, 33};
    for (int n : steps) {
        if (n < need) continue;
        if ((sps == 8 && n == 3) || (sps == 2 && n == 3) || (sps == 2 && n == 33) || (sps == 16 && n == 33)) continue;
        return n;
    }
    return 0;
}

hipError_t launch_tx_mfma(const TxParams& p, int sps, int nks, const float* bfrag, int dtype, int out_mode,
                          hipStream_t s) {
    auto go = [&](auto outt) {
        using OutT = decltype(outt);
        switch (out_mode) {
        case OUT_IQ_MIXED: return txm_sel<OUT_IQ_MIXED, OutT>(p, sps, nks, bfrag, s);
        case OUT_IQ_BASEBAND: return txm_sel<OUT_IQ_BASEBAND, OutT>(p, sps, nks, bfrag, s);
        default: return txm_sel<OUT_REAL, OutT>(p, sps, nks, bfrag, s);
        }
    };
    return dtype == 1 ? go(__half()) : go(float());
}

hipError_t launch_tx(const TxParams& p, int sps, int dtype, int out_mode, hipStream_t s) {
    return dtype == 1 ? tx_mode<__half>(p, sps, out_mode, s) : tx_mode<float>(p, sps, out_mode, s);
}

template <int DEC, typename InT, int MIX, typename OutT>
static hipError_t rx_go(const RxParams& p, hipStream_t s) {
    using C = RxCfg<DEC>;
    const int64_t ntiles = (p.nout + C::TS - 1) / C::TS;
    const size_t lds = ((size_t)DEC * rx_plane_stride(C::TS, p.K) + 1) * sizeof(float2);
    const void* k = reinterpret_cast<const void*>(&rx_fast<DEC, InT, MIX, OutT>);
    hipLaunchKernelGGL((rx_fast<DEC, InT, MIX, OutT>), dim3(persistent_grid(k, C::NT, lds, ntiles)),
                       dim3(C::NT), lds, s, p);
    return hipGetLastError();
}

template <typename InT, int MIX, typename OutT>
static hipError_t rx_dec(const RxParams& p, int decim, hipStream_t s) {
    switch (decim) {
    case 1: return rx_go<1, InT, MIX, OutT>(p, s);
    case 2: return rx_go<2, InT, MIX, OutT>(p, s);
    case 4: return rx_go<4, InT, MIX, OutT>(p, s);
    case 8: return rx_go<8, InT, MIX, OutT>(p, s);
    case 16: return rx_go<16, InT, MIX, OutT>(p, s);
    default: {
        const int64_t nblk = (p.nout + 63) / 64;
        const size_t lds = (size_t)(63 * decim + p.L) * sizeof(float2);
        hipLaunchKernelGGL((rx_generic<InT, MIX, OutT>), dim3((unsigned)(nblk > 0 ? nblk : 1)),
                           dim3(64), lds, s, p);
        return hipGetLastError();
    }
    }
}

template <typename InT, typename OutT>
static hipError_t rx_mixsel(const RxParams& p, int decim, int mix, hipStream_t s) {
    return mix == MIX_REFERENCE_REAL ? rx_dec<InT, MIX_REFERENCE_REAL, OutT>(p, decim, s)
                                     : rx_dec<InT, MIX_COMPLEX, OutT>(p, decim, s);
}

template <int DEC, int NKS, typename InT, int MIX, typename OutT>
static hipError_t rxm_go(const RxParams& p, const float* bfrag, hipStream_t s) {
    using C = RxMfmaCfg<DEC>;
    using K = RxMfma<DEC, NKS, InT, MIX, OutT>;
    const int64_t ntiles = (p.nout + C::TS - 1) / C::TS;
    const size_t lds = (size_t)K::LDS_SAMPLES * sizeof(float2) + (size_t)K::TBL * sizeof(float);
    const void* k = reinterpret_cast<const void*>(&rx_mfma<DEC, NKS, InT, MIX, OutT>);
    hipLaunchKernelGGL((rx_mfma<DEC, NKS, InT, MIX, OutT>), dim3(persistent_grid(k, C::NT, lds, ntiles)),
                       dim3(C::NT), lds, s, p, bfrag);
    return hipGetLastError();
}

template <typename InT, int MIX, typename OutT>
static hipError_t rxm_sel(const RxParams& p, int decim, int nks, const float* bfrag, hipStream_t s) {
#define RXM(D, N) if (decim == D && nks == N) return rxm_go<D, N, InT, MIX, OutT>(p, bfrag, s);
    RXM(4, 24) RXM(4, 32) RXM(4, 48) RXM(2, 16) RXM(2, 24) RXM(2, 40) RXM(8, 40) RXM(8, 48) RXM(8, 64)
#undef RXM
    return hipErrorInvalidValue;
}

int rx_mfma_ksteps(int decim, int L) {
    const int need = (15 * decim + L + 3) / 4;
    int cand[3] = {0, 0, 0};
    if (decim == 4) { cand[0] = 24; cand[1] = 32; cand[2] = 48; }
    else if (decim == 2) { cand[0] = 16; cand[1] = 24; cand[2] = 40; }
    else if (decim == 8) { cand[0] = 40; cand[1] = 48; cand[2] = 64; }
    for (int n : cand)
        if (n >= need) return n;
    return 0;
}

hipError_t launch_rx_mfma(const RxParams& p, int decim, int nks, const float* bfrag, int in_dtype,
                          int out_dtype, int mix, hipStream_t s) {
    auto go = [&](auto in_t, auto out_t) {
        using InT = decltype(in_t);
        using OutT = decltype(out_t);
        return mix == MIX_REFERENCE_REAL ? rxm_sel<InT, MIX_REFERENCE_REAL, OutT>(p, decim, nks, bfrag, s)
                                         : rxm_sel<InT, MIX_COMPLEX, OutT>(p, decim, nks, bfrag, s);
    };
    if (in_dtype == 1) return out_dtype == 1 ? go(__half(), __half()) : go(__half(), float());
    return out_dtype == 1 ? go(float(), __half()) : go(float(), float());
}

hipError_t launch_rx(const RxParams& p, int decim, int in_dtype, int out_dtype, int mix,
                     hipStream_t s) {
    if (in_dtype == 1)
        return out_dtype == 1 ? rx_mixsel<__half, __half>(p, decim, mix, s)
                              : rx_mixsel<__half, float>(p, decim, mix, s);
    return out_dtype == 1 ? rx_mixsel<float, __half>(p, decim, mix, s)
                          : rx_mixsel<float, float>(p, decim, mix, s);
}

hipError_t launch_fir(const FirParams& p, hipStream_t s) {
    const int64_t nblk = (p.N + kFirTS - 1) / kFirTS;
    const size_t lds = (size_t)(kFirTS + p.L + 1) * sizeof(float);
    hipLaunchKernelGGL(fir_real, dim3((unsigned)(nblk > 0 ? nblk : 1)), dim3(kFirNT), lds, s, p);
    return hipGetLastError();
}

hipError_t launch_prng_bits(uint64_t seed, uint8_t* out, size_t nbits, hipStream_t s) {
    const size_t words = (nbits + 63) / 64;
    const size_t nblk = (words + 255) / 256;
    if (nblk == 0) return hipSuccess;
    hipLaunchKernelGGL(prng_bits, dim3((unsigned)nblk), dim3(256), 0, s, seed, out, nbits);
    return hipGetLastError();
}

}  // namespace mk
