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

// Diagnostic builds only (-DMODEM_STAMPS, tools/stamps.py --kernel tx): s_memtime per wave at the
// phase boundaries of each TX tile (lane 0's vector store into a buffer nothing else reads).
// Layout [block * 4 + wave][tile slot 0..7][point 0..7]; slot 7: entry / realtime / HW_ID / XCC_ID
// / exit / realtime.
#ifdef MODEM_STAMPS
constexpr int kTxStampWaves = 8192, kTxStampTiles = 8, kTxStampPts = 8;
__device__ unsigned long long g_modem_tx_stamps[kTxStampWaves * kTxStampTiles * kTxStampPts];
__device__ __forceinline__ void modem_tx_stamp(int tile, int pt, unsigned long long v) {
    const int w = (int)blockIdx.x * 4 + ((int)threadIdx.x >> 6);
    if ((threadIdx.x & 63) == 0 && w < kTxStampWaves && tile < kTxStampTiles)
        g_modem_tx_stamps[((size_t)w * kTxStampTiles + tile) * kTxStampPts + pt] = v;
}
#define TX_STAMP(t, k) modem_tx_stamp((int)(t), (k), __builtin_amdgcn_s_memtime())
#else
#define TX_STAMP(t, k) ((void)0)
#endif

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
__device__ __forceinline__ float2 tx_mix(float w, uint64_t n, bool exact_idx, float2 y) {
    if (OUT_MODE == OUT_IQ_BASEBAND) return y;
    float s, c;
    sincos_phase(carrier_phase(w, n, exact_idx), s, c);
    return make_float2(y.x * c - y.y * s, y.x * s + y.y * c);
}

template <int OUT_MODE, typename OutT>
__device__ __forceinline__ void tx_emit(const TxParams& p, int64_t j, float2 y0, float2 y1,
                                        bool two) {
    const uint64_t n = p.s0 + (uint64_t)j;
    const float2 z0 = tx_mix<OUT_MODE>(p.w, n, p.exact_idx, y0);
    if (two) {
        const float2 z1 = tx_mix<OUT_MODE>(p.w, n + 1, p.exact_idx, y1);
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
        sincos_phase(carrier_phase_off(p.w, nb, off, p.exact_idx), s, c);
        z0 = make_float2(y0.x * c - y0.y * s, y0.x * s + y0.y * c);
        if (two) {
            sincos_phase(carrier_phase_off(p.w, nb, off + 1, p.exact_idx), s, c);
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
// The zero-stuffed polyphase FIR on the matrix cores (v_mfma_f32_16x16x32_f16):
//   rows i  = 16 row-blocks of SB = 16/SPS consecutive symbols,
//   cols j  = (symbol c in the block, phase p) -> sample SPS*c + p of the block (16 samples),
//   k  = o  = offset in a W = 32*NKS symbol window ending at the block's last symbol,
//   A[i][o] = a[block_i - PRE + o] (symbol values, from LDS), B[o][j] = h[p + SPS*(c + PRE - o)].
// As on the RX, every operand is split in two f16 halves (a = a_hi + a_lo, round to nearest)
// and A*B ~= A_hi*B_hi + A_hi*B_lo + A_lo*B_hi accumulates in f32 (6 MFMAs per k-step for the
// re and im rails). The LUT and the taps are scaled by exact powers of two on the host
// (2^lut_scale_exp, 2^tap_scale_exp; 0 when the maxima already lie in [2^-3, 2^15), else into
// [2^14, 2^15)), split there, and the outputs are scaled back. When every LUT component is an
// integer multiple of one scale s (QAM, BPSK at pi/4, QPSK at 0, BASK) the symbols are the
// exact f16 integer levels, s is folded into the taps and the A_lo products vanish. Row-blocks are aligned to the absolute symbol index
// (lead = symbols before this call, mod SB), so a symbol always meets the same taps at the
// same k positions and a stream cut into calls gives the same samples as one call.
// Sample-and-hold (no taps) stays on the exact VALU kernels.
template <int SPS, int SUB_> struct TxMfmaCfg {
    static constexpr int SB = 16 / SPS;          // symbols per row-block
    static constexpr int NT = 256;               // 4 waves
    static constexpr int SUB = SUB_;             // 16x16 tiles per wave per tile: 4, 1 (small calls)
    static constexpr int TS = 4 * SUB * 16 * SB; // symbols per workgroup tile
    static constexpr int NCOP = SB % 4 == 0 ? 1 : 4 / SB;   // plane copies (8-B aligned A reads)
};

// Carrier mix of one sample, packed: (re, im) = (y*cs - yi*sn, y*sn + yi*cs), y = (yr, yi),
// cssn = (cs, sn) straight from v_sin/v_cos.
__device__ __forceinline__ cf2 tx_cmix(cf2 y, cf2 cssn) {
    // vector ops (v_pk_mul_f32 + v_pk_fma_f32 with op_sel / neg modifiers): visible to the
    // compiler's hazard recognizer, which pads only where a v_sin/v_cos result is read too early
    const cf2 t = y * cssn.xx;
    return __builtin_elementwise_fma(y.yx, (cf2){-cssn.y, cssn.y}, t);
}

typedef _Float16 th8 __attribute__((ext_vector_type(8)));
typedef _Float16 th4 __attribute__((ext_vector_type(4)));

template <int SPS, int NKS, int OUT_MODE, typename OutT, int SUB_ = 4>
struct TxMfma {
    using C = TxMfmaCfg<SPS, SUB_>;
    static constexpr int SB = C::SB, NT = C::NT, SUB = C::SUB, TS = C::TS, NCOP = C::NCOP;
    static constexpr int W = 32 * NKS;             // window symbols per row-block
    static constexpr int PRE = W - SB;             // window symbols before a row-block
    static constexpr int NE = TS + PRE;            // symbols staged per tile
    static constexpr int U = (NE + NT - 1) / NT;   // staging slots per lane
    static constexpr int PLN = (NE + 3 * 4 + 7) & ~7;   // halves per plane copy
    // LDS: NCOP copies x 4 planes (re_hi, re_lo, im_hi, im_lo) of PLN halves, then the split
    // LUT (4 halves per entry)
    // Halves between plane copies. ds_read2_b64 is serviced 16 lanes at a time with bank =
    // dword mod 32 (MI355X_MICROARCH.md §LDS): with 2 copies (sps 8) the odd rows' copy must
    // sit 28 halves past a multiple of 64, else every read of a 16-lane group is 2-way
    // conflicted (8 extra LDS cycles per read; 13 M per C5 launch, PMC SQ_LDS_BANK_CONFLICT);
    // with 4 copies (sps 16) a residue of 16 halves the conflicts of 0.
    static constexpr int CRES = SB == 2 ? 28 : SB == 1 ? 16 : 0;
    static constexpr int CST = 4 * PLN + (NCOP > 1 ? (CRES - (4 * PLN) % 64 + 64) % 64 : 0);
    static constexpr int PLANES = NCOP * CST;

    // Raw bits word of symbol m, BPS bytes (fast path: aligned, no leftover bits).
    template <int BPS>
    __device__ static uint64_t load_word(const uint8_t* bits, int64_t m) {
        const uint8_t* b = bits + m * BPS;
        if (BPS == 1) return *b;
        if (BPS == 2) return *reinterpret_cast<const uint16_t*>(b);
        if (BPS == 4) return *reinterpret_cast<const uint32_t*>(b);
        return *reinterpret_cast<const uint64_t*>(b);
    }

    // Symbol e of the tile (window coordinates) into every plane copy: copy c holds symbol e
    // at half index e + c*SB, so a row-block starting at blk*SB reads copy ((-blk*SB) mod 4)/SB
    // 8-B aligned.
    __device__ static void put(_Float16* pl, int e, th4 v) {
#pragma unroll
        for (int c = 0; c < NCOP; ++c) {
            _Float16* q = pl + c * CST + e + c * SB;
            q[0] = v[0]; q[PLN] = v[1]; q[2 * PLN] = v[2]; q[3 * PLN] = v[3];
        }
    }

    // f32 symbol value -> scaled (2^ka) split halves (re_hi, re_lo, im_hi, im_lo), as the host
    // splits the LUT (round to nearest both times).
    __device__ static th4 split_value(const TxParams& p, float2 v) {
        if (p.levels)      // the exact integer level of a history symbol (lo halves zero)
            return (th4){(_Float16)__builtin_rintf(v.x * p.level_inv), (_Float16)0.0f,
                         (_Float16)__builtin_rintf(v.y * p.level_inv), (_Float16)0.0f};
        const float r = __builtin_ldexpf(v.x, p.lut_scale_exp), i = __builtin_ldexpf(v.y, p.lut_scale_exp);
        const _Float16 rh = (_Float16)r, ih = (_Float16)i;
        return (th4){rh, (_Float16)(r - (float)rh), ih, (_Float16)(i - (float)ih)};
    }

    // General staging: first tile (history), leftover bits, flush, any bps. Every lane's symbol
    // indices (and history values) are loaded first, all in flight together, then looked up in
    // the LDS copy of the split LUT (the same halves split_value gives the f32 LUT entry): the
    // per-symbol form waited for each bits load and then for a global LUT load, ~10 serialized
    // memory round trips per C3 tile.
    __device__ static void stage_slow(const TxParams& p, _Float16* pl, const th4* lut_s, int64_t ms) {
        constexpr int NK = (NE + NT - 1) / NT;
        const int tid = threadIdx.x;
        uint32_t idx[NK];
        float2 hv[NK];
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            const int e = tid + k * NT;
            const int64_t m = ms + e;
            idx[k] = 0;
            hv[k] = make_float2(0.f, 0.f);
            if (e < NE) {
                if (m < 0) { if (m >= -(int64_t)(p.K - 1)) hv[k] = p.hist[m + p.K - 1]; }
                else if (m < p.nsym_valid) idx[k] = tx_symbol_index(p, m);
            }
        }
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            const int e = tid + k * NT;
            const int64_t m = ms + e;
            if (e < NE) put(pl, e, m >= 0 && m < p.nsym_valid ? lut_s[idx[k]] : split_value(p, hv[k]));
        }
    }

    // 16x16 sub-tile q of this wave: D = sum over the window of A*B (split products).
    // LV: integer-level symbols (exact f16, no lo plane): 2 MFMAs per rail and k-step, else 3.
    template <bool LV>
    __device__ static void fir(const _Float16* pl, int q, const th8 (&bh)[NKS], const th8 (&bl)[NKS],
                               f32x4& dre, f32x4& dim) {
        const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        const int i = lane & 15, g = lane >> 4;
        const int blk = (wave * SUB + q) * 16 + i;                  // row-block in the tile
        const int cp = ((4 - ((blk * SB) & 3)) & 3) / (SB < 4 ? SB : 4);   // copy shifting the row to 8 B
        // opaque lane offset: every plane / k-step read is this base + a non-negative immediate
        int aoff = (NCOP > 1 ? cp : 0) * CST + blk * SB + (NCOP > 1 ? cp * SB : 0) + 8 * g;
        asm volatile("" : "+v"(aoff));
        const _Float16* ar = pl + aoff;
        typedef _Float16 tq4 __attribute__((ext_vector_type(4), aligned(8)));
        auto ld8 = [](const _Float16* a) {                          // 8-B aligned 16-B read
            const tq4 x = *reinterpret_cast<const tq4*>(a), y = *reinterpret_cast<const tq4*>(a + 4);
            return (th8){x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
        };
#ifdef MODEM_ABLATE_FIR
        const th8 a0 = ld8(ar);
        dre = (f32x4){(float)a0[0], 0.f, 0.f, 0.f};
        dim = (f32x4){(float)bh[0][0], 0.f, 0.f, 0.f};
        return;
#endif
        f32x4 r0 = {0.f, 0.f, 0.f, 0.f}, m0 = r0;     // one accumulator per rail
        th8 a[2][4];
        auto load = [&](int s, int slot) {
            a[slot][0] = ld8(ar + 32 * s);
            if (!LV) a[slot][1] = ld8(ar + PLN + 32 * s);
            a[slot][2] = ld8(ar + 2 * PLN + 32 * s);
            if (!LV) a[slot][3] = ld8(ar + 3 * PLN + 32 * s);
        };
        load(0, 0);
#pragma unroll
        for (int s = 0; s < NKS; ++s) {
            const int c = s & 1;
            if (s + 1 < NKS) load(s + 1, c ^ 1);
            r0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[c][0], bh[s], r0, 0, 0, 0);
            m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[c][2], bh[s], m0, 0, 0, 0);
            r0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[c][0], bl[s], r0, 0, 0, 0);
            m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[c][2], bl[s], m0, 0, 0, 0);
            if (!LV) {
                r0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[c][1], bh[s], r0, 0, 0, 0);
                m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[c][3], bh[s], m0, 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        dre = r0;
        dim = m0;
    }

    // Full 16x16 tile, carrier index < 2^53: unconditional stores. jt = call sample index of
    // the sub-tile's first sample. Per sample: packed unscale (2^-kab), bit-exact phase,
    // sin/cos, packed mix; stores through a uniform base + 32-bit lane offsets.
    __device__ static void emit_full(const TxParams& p, int64_t jt, const f32x4& dre, const f32x4& dim, cf2 unscale) {
        const int lane = threadIdx.x & 63;
        int loff = 64 * (lane >> 4) + (lane & 15);          // sample of row r: loff + 16 r
        asm volatile("" : "+v"(loff));
        const double nb = (double)(p.s0 + (uint64_t)jt) + (double)loff;
        cf2 z[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) z[r] = (cf2){dre[r], dim[r]};
        if (unscale.x != 1.0f) {                            // uniform; scale 1 is the usual case
#pragma unroll
            for (int r = 0; r < 4; ++r) z[r] *= unscale;
        }
#ifndef MODEM_ABLATE_MIX
        if (OUT_MODE != OUT_IQ_BASEBAND) {
            // rows (0, 1) and (2, 3) as two packed phase pairs, side by side
            const cf2 nf0 = (cf2){idx_f32(nb), idx_f32(nb + 16.0)};
            const cf2 nf1 = (cf2){idx_f32(nb + 32.0), idx_f32(nb + 48.0)};
            const cf2 ph0 = phase_from_f2(p.w, nf0), ph1 = phase_from_f2(p.w, nf1);
            cf2 sn0, cs0, sn1, cs1;
            sincos_phase2(ph0, sn0, cs0);
            sincos_phase2(ph1, sn1, cs1);
            z[0] = tx_cmix(z[0], (cf2){cs0.x, sn0.x});
            z[1] = tx_cmix(z[1], (cf2){cs0.y, sn0.y});
            z[2] = tx_cmix(z[2], (cf2){cs1.x, sn1.x});
            z[3] = tx_cmix(z[3], (cf2){cs1.y, sn1.y});
        }
#endif
#ifdef MODEM_ABLATE_STORE
#pragma unroll
        for (int r = 0; r < 4; ++r) asm volatile("" :: "v"(z[r]));
#else
        // wave-uniform base in SGPRs + 32-bit lane byte offsets (saddr + voffset stores)
        constexpr int SBYTES = (OUT_MODE == OUT_REAL ? 1 : 2) * (int)sizeof(OutT);
        const uint64_t oa = (uint64_t)p.out + (uint64_t)jt * SBYTES;
        char* ob = reinterpret_cast<char*>(((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(oa >> 32)) << 32) |
                                           (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)oa));
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            char* q = ob + (uint32_t)((loff + 16 * r) * SBYTES);
            if (OUT_MODE == OUT_REAL) OutIO<OutT>::store_real_one(q, 0, z[r].x);
            else OutIO<OutT>::store_one(q, 0, z[r].x, z[r].y);
        }
#endif
    }

    // Partial tile, samples before the call, or carrier index >= 2^53: guarded, 64-bit
    // indices; the same arithmetic as emit_full (a sample's bits never depend on the path).
    __device__ static void emit_edge(const TxParams& p, int64_t jt, const f32x4& dre, const f32x4& dim, cf2 unscale) {
        const int lane = threadIdx.x & 63;
        const int64_t jend = p.nsym * SPS;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int off = 16 * (4 * (lane >> 4) + r) + (lane & 15);
            if (jt + off < 0 || jt + off >= jend) continue;
            cf2 z = (cf2){dre[r], dim[r]} * unscale;
            if (OUT_MODE != OUT_IQ_BASEBAND) {
                float sn, cs;
                sincos_phase(carrier_phase_off(p.w, p.s0 + (uint64_t)jt, off, p.exact_idx), sn, cs);
                z = tx_cmix(z, (cf2){cs, sn});
            }
            if (OUT_MODE == OUT_REAL) OutIO<OutT>::store_real_one(p.out, jt + off, z.x);
            else OutIO<OutT>::store_one(p.out, jt + off, z.x, z.y);
        }
    }

    // Tiles t0, t0 + ts, ... below t1. Tile t holds symbols [t*TS - lead, (t+1)*TS - lead) of the call. BPS > 0: bits aligned,
    // no leftover bits, carrier index < 2^53 (the steady state); BPS == 0: general path only.
    template <int BPS>
    __device__ static void run(const TxParams& p, _Float16* pl, th4* lut_s, const th8 (&bh)[NKS],
                               const th8 (&bl)[NKS], int64_t t0, int64_t t1, int64_t ts) {
        const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        const int lead = p.lead;
        const int kab = p.lut_scale_exp + p.tap_scale_exp;
        const bool lv = p.levels != 0;
        const float us = __builtin_ldexpf(1.0f, -kab);             // exact (|kab| < 126)
        const cf2 unscale = {us, us};
        const int64_t mlast = p.nsym_valid - 1;
        // full tile: every staged symbol is data of this call, every sample is emitted
        auto full = [&](int64_t t) {
            const int64_t ms = t * TS - lead - PRE;
            return BPS > 0 && ms >= 0 && ms + NE <= p.nsym_valid && t * TS - lead + TS <= p.nsym;
        };
        uint64_t pre[U];
        auto prefetch = [&](int64_t t) {
            const int64_t ms = t * TS - lead - PRE;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                int64_t m = ms + tid + NT * u;
                m = m < 0 ? 0 : (m > mlast ? mlast : m);
                pre[u] = load_word<BPS>(p.bits, m);
            }
        };
        int64_t t = t0;
        // the first tile's bits are requested before the LUT goes to LDS, so that the two
        // memory latencies at the kernel's start overlap
        TX_STAMP(7, 0);
        bool ready = t < t1 && full(t);
        if (ready) prefetch(t);
        const th4* lut_h = reinterpret_cast<const th4*>(p.lut_h);
        for (int i = tid; i < (1 << p.bps); i += NT) lut_s[i] = lut_h[i];
        __syncthreads();   // LUT visible
#ifdef MODEM_STAMPS
        modem_tx_stamp(7, 1, __builtin_amdgcn_s_memrealtime());
        modem_tx_stamp(7, 2, __builtin_amdgcn_s_getreg((31 << 11) | 4));    // HW_ID
        modem_tx_stamp(7, 3, __builtin_amdgcn_s_getreg((31 << 11) | 20));   // XCC_ID
        int si = 0;
#endif
        while (t < t1) {
            if (full(t)) {
                if (!ready) prefetch(t);
                ready = false;
                for (; t < t1 && full(t); t += ts) {
#ifdef MODEM_STAMPS
                    TX_STAMP(si, 0);
#endif
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int e = tid + NT * u;
                        if (e < NE) put(pl, e, lut_s[word_index(pre[u], BPS)]);
                    }
#ifdef MODEM_STAMPS
                    TX_STAMP(si, 1);
#endif
                    __syncthreads();
#ifdef MODEM_STAMPS
                    TX_STAMP(si, 2);
#endif
                    if (t + ts < t1) prefetch(t + ts);   // next bits fly during the MFMAs
                    const int64_t j0 = (t * TS - lead) * SPS;
#pragma unroll
                    for (int q = 0; q < SUB; ++q) {
                        f32x4 dre, dim;
                        if (lv) fir<true>(pl, q, bh, bl, dre, dim);
                        else fir<false>(pl, q, bh, bl, dre, dim);
                        // the epilogue (carrier phase, sin/cos, mix, stores) issues ahead
                        // of the other workgroups' staging and filter: +0.6 % C3 bench in
                        // three interleaved pairs (profiles/r02_store_layout_ab.txt)
                        __builtin_amdgcn_s_setprio(1);
                        emit_full(p, j0 + ((int64_t)(wave * SUB + q) * 16 * SB) * SPS, dre, dim, unscale);
                        __builtin_amdgcn_s_setprio(0);
                    }
#ifdef MODEM_STAMPS
                    TX_STAMP(si, 4);
#endif
                    __syncthreads();                     // the window is restaged next trip
#ifdef MODEM_STAMPS
                    TX_STAMP(si, 5);
                    ++si;
#endif
                }
            } else {
#ifdef MODEM_STAMPS
                TX_STAMP(si, 6);
#endif
                stage_slow(p, pl, lut_s, t * TS - lead - PRE);
                __syncthreads();
                const int64_t j0 = (t * TS - lead) * SPS;
#pragma unroll 1
                for (int q = 0; q < SUB; ++q) {
                    f32x4 dre, dim;
                    if (lv) fir<true>(pl, q, bh, bl, dre, dim);
                    else fir<false>(pl, q, bh, bl, dre, dim);
                    emit_edge(p, j0 + ((int64_t)(wave * SUB + q) * 16 * SB) * SPS, dre, dim, unscale);
                }
                __syncthreads();
#ifdef MODEM_STAMPS
                TX_STAMP(si, 7);
                ++si;
#endif
                t += ts;
            }
        }
        TX_STAMP(7, 4);
#ifdef MODEM_STAMPS
        modem_tx_stamp(7, 5, __builtin_amdgcn_s_memrealtime());
#endif
    }
};

// One channel's share of a launch: workgroup `bid` of `nb` working on channel p.
template <int SPS, int NKS, int OUT_MODE, typename OutT, int SUB>
__device__ __forceinline__ void tx_mfma_body(const TxParams& p, const th8* __restrict__ bfrag,
                                             int64_t bid, int64_t nb) {
    using K = TxMfma<SPS, NKS, OUT_MODE, OutT, SUB>;
    extern __shared__ __attribute__((aligned(16))) _Float16 lds_t[];
    _Float16* pl = lds_t;
    th4* lut_s = reinterpret_cast<th4*>(lds_t + K::PLANES);
    const int tid = threadIdx.x, lane = tid & 63;
    if (bid == 0) tx_state_update(p);
    th8 bh[NKS], bl[NKS];                        // this lane's B fragments (hi, lo) per k-step
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
        bh[s] = bfrag[(2 * s) * 64 + lane];
        bl[s] = bfrag[(2 * s + 1) * 64 + lane];
    }
    const int64_t ntiles = (p.nsym + p.lead + K::TS - 1) / K::TS;
    // tiles bid, bid + nb, ...: concurrently running workgroups work on neighbouring tiles
    // (measured 1 % faster on C3 than contiguous ranges per workgroup)
    const int64_t t0 = bid, t1 = ntiles, ts = nb;
    if (t0 >= t1) return;
    if (p.fast_bits && p.exact_idx) {              // one uniform switch: the tile loop is specialised
        switch (p.bps) {
        case 1: K::template run<1>(p, pl, lut_s, bh, bl, t0, t1, ts); return;
        case 2: K::template run<2>(p, pl, lut_s, bh, bl, t0, t1, ts); return;
        case 4: K::template run<4>(p, pl, lut_s, bh, bl, t0, t1, ts); return;
        case 8: K::template run<8>(p, pl, lut_s, bh, bl, t0, t1, ts); return;
        }
    }
    K::template run<0>(p, pl, lut_s, bh, bl, t0, t1, ts);
}

template <int SPS, int NKS, int OUT_MODE, typename OutT, int SUB>
__global__ __launch_bounds__(256) void tx_mfma(const TxParams p, const th8* __restrict__ bfrag) {
    tx_mfma_body<SPS, NKS, OUT_MODE, OutT, SUB>(p, bfrag, blockIdx.x, gridDim.x);
}

// A batch of independent channels of one configuration (modem_tx_process_batch): workgroup
// b serves channel b / g as its workgroup b % g of g.
template <int SPS, int NKS, int OUT_MODE, typename OutT, int SUB>
__global__ __launch_bounds__(256) void tx_mfma_batch(const TxBatch b, const th8* __restrict__ bfrag) {
    const int ch = (int)(blockIdx.x / (unsigned)b.g);
    const unsigned bid = blockIdx.x - (unsigned)ch * b.g;
    const TxParams p = b.p[ch];     // one bulk copy: the body's uses read registers, not kernarg
    tx_mfma_body<SPS, NKS, OUT_MODE, OutT, SUB>(p, bfrag, bid, b.g);
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
        const float* tq = p.taps_q ? p.taps_q : p.taps;   // EvenOddOffset: Q rail delayed
        for (int t = 0; t < K; ++t) {
            const float2 a = lds[ml - t + K - 1];
            yr = __builtin_fmaf(a.x, p.taps[t * SPS + q], yr);
            yi = __builtin_fmaf(a.y, tq[t * SPS + q], yi);
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

// ------------------------------------------------------- sample-dependent phasors ----
// DigitalModulator (modulator.rs:85-100) with a phasor whose (i, q) depend on more than the
// symbol's bits, one thread per sample, sample-and-hold:
//   DCQPSK (dcqpsk.rs:23-52): the term alternates between MAP + pi/4 and MAP at every symbol
//     tick (update() toggles `even` before the first symbol) -> host table of 2 x 4 entries
//     indexed by the parity of the symbol count since the stream start;
//   CPFSK (cpfsk.rs:27-45): amp * cos/sin(2*sym * freq * s);
//   MSK (msk.rs:23-37, over EvenOddOffset when q_off = sps/2): amp * sign(b0) * cos(pi/2*s/spb),
//     -amp * sign(b1) * sin(pi/2*s/spb);
// s is the carrier sample index after Carrier::next (sample n -> s0 + n + 1), converted like
// Rust's `as f32`; f32 operations in the reference's left-to-right order.
enum { PH_DCQPSK = 8, PH_DMPSK = 9, PH_CPFSK = 10, PH_MSK = 11, PH_MFSK = 12, PH_BFSK = 13 };

// mod_trig (util.rs:3-6) with the IEEE quotient, for any finite f32 (the scan's phases can be
// negative, where the carrier's shortcut is not proven).
__device__ __forceinline__ float mod_trig_ieee(float x) {
#pragma clang fp contract(off)
    return x - kTwoPi * __builtin_floorf(x / kTwoPi);
}

// DMPSK / MFSK / BFSK: update() runs at every symbol tick (modulator.rs:90-93) with the
// phase carried in f32 from symbol to symbol, so the states are a serial recurrence. One
// workgroup: its lanes decode 256 symbol indices at a time into LDS, lane 0 runs the
// recurrence exactly as the reference does, and the lanes write the states out.
//   DMPSK (dmpsk.rs:29-33): phase = mod_trig(phase + sym * shift)
//   MFSK (mfsk.rs:68-75):   off = mod_trig(off + (cur - next) * dev * s); cur = next
//   BFSK (bfsk.rs:42-53):   on a change of bit, phase = mod_trig(phase + (b ? -dev*s : dev*(s-1)))
// s is the carrier sample index after Carrier::next at the symbol's first sample.
__global__ __launch_bounds__(256) void tx_scan(const TxParams p) {
#pragma clang fp contract(off)
    __shared__ uint32_t sidx[256];
    __shared__ float2 sst[256];
    float2 st = p.hist[0];
    for (int64_t base = 0; base < p.nsym; base += 256) {
        const int64_t m = base + threadIdx.x;
        if (m < p.nsym) sidx[threadIdx.x] = tx_symbol_index(p, m);
        __syncthreads();
        if (threadIdx.x == 0) {
            const int cnt = (int)(p.nsym - base < 256 ? p.nsym - base : 256);
            for (int j = 0; j < cnt; ++j) {
                const uint32_t idx = sidx[j];
                const uint64_t su = p.s0 + (uint64_t)(base + j) * (uint64_t)p.sps + 1u;
                if (p.ph_kind == PH_DMPSK) {
                    st.x = mod_trig_ieee(st.x + (float)idx * p.ph_shift);
                } else if (p.ph_kind == PH_MFSK) {
                    const float next = p.ph_map ? (float)(2 * (int)idx) : (float)(2 * (int)idx - (int)p.ph_max);
                    st.y = st.y + (st.x - next) * p.ph_freq * (float)su;
                    st.y = mod_trig_ieee(st.y);
                    st.x = next;
                } else {                                   // BFSK: st = (phase, prev bit)
                    const float b = (float)(idx & 1u);
                    if (b != st.y) {
                        const float d = b == 1.0f ? -(p.ph_freq * (float)su) : p.ph_freq * (float)(su - 1u);
                        st.x = mod_trig_ieee(st.x + d);
                        st.y = b;
                    }
                }
                sst[j] = st;
            }
        }
        __syncthreads();
        if (m < p.nsym) p.scan[m] = sst[threadIdx.x];
        __syncthreads();
    }
    if (threadIdx.x == 0) p.hist_new[0] = st;
}

__device__ __forceinline__ float2 tx_phasor_value(const TxParams& p, int64_t n, int64_t m) {
#pragma clang fp contract(off)
    const uint32_t idx = tx_symbol_index(p, m);
    const float sf = (float)(p.s0 + (uint64_t)n + 1u);
    if (p.ph_kind == PH_DCQPSK) return p.lut[(((p.sym0 + (uint64_t)m) & 1u) ? 4u : 0u) + idx];
    if (p.ph_kind == PH_DMPSK || p.ph_kind == PH_MFSK || p.ph_kind == PH_BFSK) {
        const float2 st = p.scan[m];
        float x;
        if (p.ph_kind == PH_DMPSK) x = st.x;                                  // dmpsk.rs:35-41
        else if (p.ph_kind == PH_MFSK) x = st.x * p.ph_freq * sf + st.y;      // mfsk.rs:61-63
        else x = (float)(idx & 1u) * p.ph_freq * sf + st.x;                   // bfsk.rs:22-28
        float sn, cs;
        sincosf(x, &sn, &cs);
        return make_float2(p.ph_amp * cs, p.ph_amp * sn);
    }
    if (p.ph_kind == PH_CPFSK) {
        const float x = (2.0f * (float)idx) * p.ph_freq * sf;
        float sn, cs;
        sincosf(x, &sn, &cs);
        return make_float2(p.ph_amp * cs, p.ph_amp * sn);
    }
    // MSK: I bit from this symbol, Q bit from the symbol q_off samples earlier
    uint32_t qidx = idx;
    if (p.q_off) {
        const int64_t mq = (n - p.q_off) >= 0 ? (n - p.q_off) / p.sps : -1;
        qidx = mq >= 0 ? tx_symbol_index(p, mq) : (uint32_t)p.hist[0].x;
    }
    const float x = 1.57079637f * sf / (float)p.ph_spb;          // PI / 2.0 * s / spb
    float sn, cs;
    sincosf(x, &sn, &cs);
    const float si = ((idx >> 1) & 1u) ? 1.0f : -1.0f, sq = (qidx & 1u) ? 1.0f : -1.0f;
    return make_float2(p.ph_amp * si * cs, -p.ph_amp * sq * sn);
}

template <int OUT_MODE, typename OutT>
__global__ __launch_bounds__(256) void tx_phasor(const TxParams p) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        // state for the next call: the last symbol's index (the offset Q rail; the scanned
        // phasors' state comes from tx_scan), leftover bits
        if (p.scan == nullptr)
            p.hist_new[0] = p.nsym > 0 ? make_float2((float)tx_symbol_index(p, p.nsym - 1), 0.f) : p.hist[0];
        if (p.update_carry)
            for (int i = 0; i < p.ncarry_new; ++i) {
                const int64_t l = p.nsym * p.bps + i;
                p.carry_new[i] = l < p.ncarry ? p.carry[l] : p.bits[l - p.ncarry];
            }
    }
    const int64_t nsamp = p.nsym * p.sps;
    for (int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; n < nsamp;
         n += (int64_t)gridDim.x * blockDim.x) {
        const float2 y = tx_phasor_value(p, n, n / p.sps);
        tx_emit<OUT_MODE, OutT>(p, n, y, make_float2(0.f, 0.f), false);
    }
}

hipError_t launch_tx_phasor(const TxParams& p, int dtype, int out_mode, hipStream_t s) {
    const int64_t nsamp = p.nsym * p.sps;
    if (p.scan != nullptr) {
        hipLaunchKernelGGL(tx_scan, dim3(1), dim3(256), 0, s, p);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((nsamp + 255) / 256, 8192));
    auto go = [&](auto outt) {
        using OutT = decltype(outt);
        switch (out_mode) {
        case OUT_IQ_MIXED: hipLaunchKernelGGL((tx_phasor<OUT_IQ_MIXED, OutT>), dim3(grid), dim3(256), 0, s, p); break;
        case OUT_IQ_BASEBAND: hipLaunchKernelGGL((tx_phasor<OUT_IQ_BASEBAND, OutT>), dim3(grid), dim3(256), 0, s, p); break;
        default: hipLaunchKernelGGL((tx_phasor<OUT_REAL, OutT>), dim3(grid), dim3(256), 0, s, p); break;
        }
        return hipGetLastError();
    };
    return dtype == 1 ? go(__half()) : go(float());
}

template <int OM, typename OutT>
static hipError_t tx_sps(const TxParams& p, int sps, hipStream_t s) {
    switch (p.taps_q ? 0 : sps) {                  // a delayed Q rail: generic kernel
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

// Tile size by the work: 4 sub-tiles per wave when the call has at least four such tiles
// per CU, else one (a small call, C2: 2^18 symbols, then still spreads over every SIMD). The
// 16x16 sub-tiles are computed alike either way: results do not depend on the choice.
inline bool tx_small_tiles(int64_t nsym, int sb) { return nsym < (int64_t)4 * 4 * 4 * 16 * sb * device_cus(); }

template <int SPS, int NKS, int OM, typename OutT, int SUB>
static hipError_t txm_go_sub(const TxParams& p, const void* bfrag, hipStream_t s) {
    using K = TxMfma<SPS, NKS, OM, OutT, SUB>;
    const int64_t ntiles = (p.nsym + p.lead + K::TS - 1) / K::TS;
    const size_t lds = (size_t)K::PLANES * 2 + ((size_t)1 << p.bps) * 8;
    const void* k = reinterpret_cast<const void*>(&tx_mfma<SPS, NKS, OM, OutT, SUB>);
    hipLaunchKernelGGL((tx_mfma<SPS, NKS, OM, OutT, SUB>), dim3(persistent_grid(k, K::NT, lds, ntiles)),
                       dim3(K::NT), lds, s, p, static_cast<const th8*>(bfrag));
    return hipGetLastError();
}
template <int SPS, int NKS, int OM, typename OutT>
static hipError_t txm_go(const TxParams& p, const void* bfrag, hipStream_t s) {
    return tx_small_tiles(p.nsym, 16 / SPS) ? txm_go_sub<SPS, NKS, OM, OutT, 1>(p, bfrag, s)
                                            : txm_go_sub<SPS, NKS, OM, OutT, 4>(p, bfrag, s);
}
template <int SPS, int NKS, int OM, typename OutT, int SUB>
static hipError_t txm_go_batch_sub(TxBatch b, const void* bfrag, hipStream_t s) {
    using K = TxMfma<SPS, NKS, OM, OutT, SUB>;
    int64_t ntiles = 0;
    for (int c = 0; c < b.nch; ++c) {
        const int64_t t = (b.p[c].nsym + b.p[c].lead + K::TS - 1) / K::TS;
        ntiles = t > ntiles ? t : ntiles;
    }
    const size_t lds = (size_t)K::PLANES * 2 + ((size_t)1 << b.p[0].bps) * 8;
    const void* k = reinterpret_cast<const void*>(&tx_mfma_batch<SPS, NKS, OM, OutT, SUB>);
    const int64_t cap = persistent_grid(k, K::NT, lds, INT64_MAX);
    int64_t g = cap / b.nch;
    g = g < 1 ? 1 : g > ntiles ? (ntiles > 0 ? ntiles : 1) : g;
    b.g = (int32_t)g;
    hipLaunchKernelGGL((tx_mfma_batch<SPS, NKS, OM, OutT, SUB>), dim3((unsigned)(g * b.nch)), dim3(K::NT), lds, s, b,
                       static_cast<const th8*>(bfrag));
    return hipGetLastError();
}
template <int SPS, int NKS, int OM, typename OutT>
static hipError_t txm_go_batch(TxBatch b, const void* bfrag, hipStream_t s) {
    int64_t nsym = 0;
    for (int c = 0; c < b.nch; ++c) nsym += b.p[c].nsym;
    return tx_small_tiles(nsym, 16 / SPS) ? txm_go_batch_sub<SPS, NKS, OM, OutT, 1>(b, bfrag, s)
                                          : txm_go_batch_sub<SPS, NKS, OM, OutT, 4>(b, bfrag, s);
}

// (sps, k-steps) variants: W = 32 * nks >= 16/sps + K - 1 symbols (K = taps per phase).
#ifdef MODEM_DEV_MIN      // experiment builds: the C2, C3 and C5 variants only
#define TXM_TABLE(X) X(4, 1) X(4, 2) X(8, 3)    // C2, C3, C5
#else
#define TXM_TABLE(X) X(2, 1) X(2, 2) X(2, 3) X(2, 5) X(4, 1) X(4, 2) X(4, 3) X(4, 5) X(4, 9) \
                     X(8, 1) X(8, 2) X(8, 3) X(8, 5) X(8, 9) X(16, 1) X(16, 2) X(16, 3) X(16, 5)
#endif

template <int OM, typename OutT>
static hipError_t txm_sel(const TxParams& p, int sps, int nks, const void* bfrag, hipStream_t s) {
#define TXM(S, N) if (sps == S && nks == N) return txm_go<S, N, OM, OutT>(p, bfrag, s);
    TXM_TABLE(TXM)
#undef TXM
    return hipErrorInvalidValue;
}

template <typename OutT>
static hipError_t txm_sel_batch(const TxBatch& b, int sps, int nks, const void* bfrag, hipStream_t s) {
#define TXM(S, N) if (sps == S && nks == N) return txm_go_batch<S, N, OUT_IQ_MIXED, OutT>(b, bfrag, s);
    TXM_TABLE(TXM)
#undef TXM
    return hipErrorInvalidValue;
}

hipError_t launch_tx_mfma_batch(const TxBatch& b, int sps, int nks, const void* bfrag, int dtype,
                                hipStream_t s) {
    if (b.nch < 1 || b.nch > kBatchMax) return hipErrorInvalidValue;
#ifdef MODEM_DEV_MIN
    if (dtype != 0) return hipErrorInvalidValue;
    return txm_sel_batch<float>(b, sps, nks, bfrag, s);
#endif
    return dtype == 1 ? txm_sel_batch<__half>(b, sps, nks, bfrag, s) : txm_sel_batch<float>(b, sps, nks, bfrag, s);
}

int tx_mfma_ksteps(int sps, int K) {
    if (sps != 2 && sps != 4 && sps != 8 && sps != 16) return 0;
    const int need = (16 / sps + K - 1 + 31) / 32;
    int best = 0;
#define TXK(S, N) if (sps == S && N >= need && (best == 0 || N < best)) best = N;
    TXM_TABLE(TXK)
#undef TXK
    return best;
}

hipError_t launch_tx_mfma(const TxParams& p, int sps, int nks, const void* bfrag, int dtype, int out_mode,
                          hipStream_t s) {
#ifdef MODEM_DEV_MIN
    if (dtype != 0 || out_mode != OUT_IQ_MIXED) return hipErrorInvalidValue;
    return txm_sel<OUT_IQ_MIXED, float>(p, sps, nks, bfrag, s);
#endif
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
#ifdef MODEM_DEV_MIN
    return hipErrorInvalidValue;
#endif
    return dtype == 1 ? tx_mode<__half>(p, sps, out_mode, s) : tx_mode<float>(p, sps, out_mode, s);
}


}  // namespace mk

#ifdef MODEM_STAMPS
// Diagnostic builds only: copy (and optionally clear) the TX stamp buffer (tools/stamps.py).
extern "C" int modem_debug_tx_stamps(void* dst, size_t bytes, int clear) {
    const size_t n = sizeof(mk::g_modem_tx_stamps);
    if (dst && hipMemcpyFromSymbol(dst, HIP_SYMBOL(mk::g_modem_tx_stamps), bytes < n ? bytes : n, 0,
                                   hipMemcpyDeviceToHost) != hipSuccess) return -1;
    if (clear) {
        void* a = nullptr;
        if (hipGetSymbolAddress(&a, HIP_SYMBOL(mk::g_modem_tx_stamps)) != hipSuccess) return -2;
        if (hipMemset(a, 0, n) != hipSuccess) return -3;
    }
    return hipDeviceSynchronize() == hipSuccess ? (int)(n / 8) : -4;
}
#endif
