// rust-modem_amd/csrc/modem_tx.hip — gfx950 TX kernels (modulator.rs:64-101 + fir.rs:18-34 +
// modulator.rs:45-48): bits -> symbol index -> LUT -> polyphase RRC -> carrier mix.
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
#include "modem_device.h"

namespace mk {

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
        // Address clamped into the call's bits. Issued only when this workgroup has a next tile
        // (a wasted tile per persistent workgroup is +25 % traffic); the stores after it stay
        // unconditional, so the next trip's vmcnt waits remain counted.
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
            if (t + 1 < tf) prefetch(m0 + TS);       // next bits fly during the MFMAs
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


}  // namespace mk
