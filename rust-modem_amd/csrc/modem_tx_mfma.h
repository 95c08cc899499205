// rust-modem_amd/csrc/modem_tx_mfma.h — the TX pulse-shaping FIR on the matrix cores (TxMfma,
// tx_mfma_body) and the symbol-mapping helpers it shares with the other TX kernels: included
// by modem_tx.hip (tx_mfma, tx_mfma_batch) and modem_chain.hip (the fused TX->RX period).
#pragma once
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
__device__ inline void tx_state_update(const TxParams& p) {
    for (int i = threadIdx.x; i < p.K - 1; i += blockDim.x)
        p.hist_new[i] = tx_symbol_value(p, p.nsym - (p.K - 1) + i);
    if (p.update_carry) {
        for (int i = threadIdx.x; i < p.ncarry_new; i += blockDim.x) {
            const int64_t l = p.nsym * p.bps + i;
            p.carry_new[i] = l < p.ncarry ? p.carry[l] : p.bits[l - p.ncarry];
        }
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
    // 16x16 tiles per wave per tile: 4, 1 (small calls); at sps 8, 8 (round 5):
    // 1024-symbol tiles like sps 4's, so the 94-symbol window halo is 8 % of the staged symbols
    // instead of 16 %, and a TX tile is exactly one RX tile (8192 samples), written on the XCD that
    // reads it back. C5 chain 259 -> 245.6 us (the RX in the chain 154.3 -> 142.8), C5 f16 175.2 ->
    // 169.2 us (profiles/r05_tx_wide.txt).
    static constexpr int SUB = SUB_ == 4 && SPS == 8 ? 8 : SUB_;
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

// An LDS copy of the samples a workgroup emits (the fused small call, modem_chain.hip: its RX
// reads them there instead of from HBM): sample j of the call at p[raw_pos(j - base)],
// 0 <= j - base < n (n a multiple of 4).
struct RawOut {
    float2* p;
    int64_t base;
    int n;
};

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
    // f16 samples out (the f16 storage sweep, tolerance 2^-10): the taps' f16 roundings only (the
    // lo B fragments carry bits below the f16 output's precision: +2^-12.2 of max|y| before the
    // output rounding on C5, tests/test_gpu_range.py), 2 MFMAs per rail and k-step instead of 3
    // (4 instead of 6 with a lo symbol plane).
    static constexpr bool HI = std::is_same<OutT, __half>::value;

    // Raw bits word of symbol m, BPS bytes (fast path: aligned, no leftover bits), in 32 bits up to
    // 4 bytes: held as 64 bits, a 1- or 2-byte word was masked (v_and) right after its load, which
    // made the tile loop's bits prefetch wait for itself at once (BPSK, QPSK).
    template <int BPS> using Word = typename std::conditional<BPS == 8, uint64_t, uint32_t>::type;
    template <int BPS>
    __device__ static Word<BPS> load_word_rsrc(__amdgpu_buffer_rsrc_t r, int off) {
        if constexpr (BPS == 1) return __builtin_amdgcn_raw_buffer_load_b8(r, off, 0, 0);
        else if constexpr (BPS == 2) return __builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0);
        else if constexpr (BPS == 4) return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
        else return __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
    }
    template <int BPS>
    __device__ static Word<BPS> load_word(const uint8_t* bits, int64_t m) {
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

    // The tile's symbols from the prefetched bits words: every slot's LUT entry read first, then the
    // plane writes (one LDS round trip for all slots; per slot, each write waited for its own read).
    // Slots wholly inside the window need no guard: only the last can reach past it (its clamped
    // word still indexes the LUT).
    template <int BPS>
    __device__ __forceinline__ static void put_all(_Float16* pl, const th4* lut_s, const Word<BPS> (&pre)[U]) {
        const int tid = threadIdx.x;
        th4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = lut_s[word_index(pre[u], BPS)];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = tid + NT * u;
            if ((u + 1) * NT <= NE || e < NE) put(pl, e, v[u]);
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
    // (e_lo > 0: only the window's symbols from e_lo on, for the sub-tiles that read no others)
    __device__ __forceinline__ static void stage_slow(const TxParams& p, _Float16* pl, const th4* lut_s, int64_t ms, int e_lo = 0) {
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
            if (e < NE && e >= e_lo) {
                if (m < 0) { if (m >= -(int64_t)(p.K - 1)) hv[k] = p.hist[m + p.K - 1]; }
                else if (m < p.nsym_valid) idx[k] = tx_symbol_index(p, m);
            }
        }
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            const int e = tid + k * NT;
            const int64_t m = ms + e;
            if (e < NE && e >= e_lo) put(pl, e, m >= 0 && m < p.nsym_valid ? lut_s[idx[k]] : split_value(p, hv[k]));
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
            if (!HI) {
                r0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[c][0], bl[s], r0, 0, 0, 0);
                m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[c][2], bl[s], m0, 0, 0, 0);
            }
            if (!LV) {
                r0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[c][1], bh[s], r0, 0, 0, 0);
                m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[c][3], bh[s], m0, 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        dre = r0;
        dim = m0;
    }

    // Full 16x16 tile, carrier index < 2^46 (TxParams::idx46): unconditional stores. jt = call
    // sample index of the sub-tile's first sample. Per sample: packed unscale (2^-kab), bit-exact
    // phase, sin/cos, packed mix; stores through a uniform base + 32-bit lane offsets.
    template <bool RAW = false, bool NT = false>
    __device__ static void emit_full(const TxParams& p, int64_t jt, const f32x4& dre, const f32x4& dim, cf2 unscale,
                                     const RawOut& ro = RawOut{}) {
        const int lane = threadIdx.x & 63;
        int loff = 64 * (lane >> 4) + (lane & 15);          // sample of row r: loff + 16 r
        asm volatile("" : "+v"(loff));
        cf2 z[4];
        // the 2^-kab unscale always (exact; a multiply by 1 when kab = 0): as a uniform branch the
        // compiler computed both sides and selected per register, 16 extra VALU per sub-tile
#pragma unroll
        for (int r = 0; r < 4; ++r) z[r] = (cf2){dre[r], dim[r]} * unscale;
        if (OUT_MODE != OUT_IQ_BASEBAND) {
            // `n as f32` of the sub-tile's samples n = n0 + loff + 16 r, n0 = s0 + jt (< 2^53 here):
            // n0 = A + b with A a multiple of 2^sh exactly representable in f32 (sh from n0's top
            // bit) and b < 2^23, so fl(A + (b + e)) — b + e an exact f32 integer — is the correctly
            // rounded index (as RxMfma::idx_split): 2 packed adds per 4 samples instead of the f64
            // index's 7 f64 operations and 4 conversions.
            const uint64_t n0 = p.s0 + (uint64_t)jt;
            const int eb = 63 - __builtin_clzll((n0 + 256) | 1);
            const int sh = eb > 23 ? eb - 23 : 0;
            const uint64_t A = n0 & ~((1ull << sh) - 1);
            const float af = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(
                __builtin_bit_cast(uint32_t, __builtin_ldexpf((float)(uint32_t)(A >> sh), sh))));
            const float bl = (float)((uint32_t)(n0 - A) + (uint32_t)loff);
            // rows (0, 1) and (2, 3) as two packed phase pairs, side by side
            const cf2 nf0 = ((cf2){bl, bl} + (cf2){0.f, 16.f}) + af;
            const cf2 nf1 = ((cf2){bl, bl} + (cf2){32.f, 48.f}) + af;
            const cf2 ph0 = phase_from_f2(p.w, nf0), ph1 = phase_from_f2(p.w, nf1);
            cf2 sn0, cs0, sn1, cs1;
            sincos_phase2(ph0, sn0, cs0);
            sincos_phase2(ph1, sn1, cs1);
            z[0] = tx_cmix(z[0], (cf2){cs0.x, sn0.x});
            z[1] = tx_cmix(z[1], (cf2){cs0.y, sn0.y});
            z[2] = tx_cmix(z[2], (cf2){cs1.x, sn1.x});
            z[3] = tx_cmix(z[3], (cf2){cs1.y, sn1.y});
        }
        if constexpr (RAW) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t i = jt + loff + 16 * r - ro.base;
                if (i >= 0 && i < ro.n) ro.p[raw_pos(i)] = make_float2(z[r].x, z[r].y);
            }
        }
        // The sub-tile's 256 samples through a buffer descriptor at its wave-uniform first sample
        // (lane byte offsets < 256 samples): buffer stores count in vmcnt only (a store through a
        // generic pointer is a flat_store, also counted in lgkmcnt, and made every later LDS wait a
        // wait for all the wave's sample stores). Every store here is unconditional and its cache
        // policy (NT: non-temporal, past the Infinity Cache, tx_nt_below) a template constant: a
        // store under a runtime branch (the policy, or the f16 form by the output's alignment) made
        // the compiler's wait tracking lose count of the stores in the tile loop, so that each
        // tile's staging waited for all of the previous tile's stores to complete.
        constexpr int SBYTES = (OUT_MODE == OUT_REAL ? 1 : 2) * (int)sizeof(OutT);
        constexpr int POL = NT && OUT_MODE != OUT_REAL ? BUF_NT : BUF_DEFAULT;
        const __amdgpu_buffer_rsrc_t rs = buf_rsrc(reinterpret_cast<const char*>(p.out) + jt * SBYTES, 256 * SBYTES);
        if constexpr (std::is_same<OutT, __half>::value && OUT_MODE != OUT_REAL) {
            // f16 samples (4 B): a lane's one-sample stores would leave every 16-lane group
            // writing half a 128-B line. Neighbour lanes swap one packed sample (DPP) so that the
            // even lane holds samples i, i+1 of row r and the odd one samples i-1, i of row r+1:
            // each 8-B store instruction then writes rows r and r+1 of the group, one whole line.
            // Every such store lands at out + 8 k: the caller guarantees an 8-byte aligned output
            // (fast_ok; a 4-byte aligned f16 buffer, a sliced (n, 2) tensor, takes emit_edge).
            const bool odd = lane & 1;
#pragma unroll
            for (int r = 0; r < 4; r += 2) {
                const uint32_t a = __builtin_bit_cast(uint32_t, __floats2half2_rn(z[r].x, z[r].y));
                const uint32_t b = __builtin_bit_cast(uint32_t, __floats2half2_rn(z[r + 1].x, z[r + 1].y));
                const uint32_t recv = (uint32_t)__builtin_amdgcn_mov_dpp((int)(odd ? a : b), 0xB1, 0xF, 0xF, false);
                const gv2u v = odd ? (gv2u){recv, b} : (gv2u){a, recv};
                const int vo = (odd ? loff + 16 * (r + 1) - 1 : loff + 16 * r) * SBYTES;
                __builtin_amdgcn_raw_buffer_store_b64(v, rs, vo, 0, POL);
            }
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int vo = (loff + 16 * r) * SBYTES;
                if constexpr (OUT_MODE == OUT_REAL) {
                    if constexpr (std::is_same<OutT, float>::value)
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, z[r].x), rs, vo, 0, POL);
                    else
                        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, __float2half_rn(z[r].x)), rs, vo, 0, POL);
                } else {
                    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(gv2u, z[r]), rs, vo, 0, POL);
                }
            }
        }
    }

    // The fast tile loop's precondition beyond the bits layout: an f16 output 8-byte aligned (its
    // pair stores, emit_full; 8 | out + 4 * SPS * k for every sub-tile since SPS is even).
    __device__ static bool out_ok(const TxParams& p) {
        return !(std::is_same<OutT, __half>::value && OUT_MODE != OUT_REAL) || ((uintptr_t)p.out & 7) == 0;
    }

    // Partial tile, samples before the call, or carrier index >= 2^53: guarded, 64-bit
    // indices; the same arithmetic as emit_full (a sample's bits never depend on the path).
    // STORE false: the LDS window only (a tail sub-tile its owner stores).
    template <bool RAW = false, bool STORE = true>
    __device__ static void emit_edge(const TxParams& p, int64_t jt, const f32x4& dre, const f32x4& dim, cf2 unscale,
                                     const RawOut& ro = RawOut{}) {
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
            if constexpr (RAW) {
                const int64_t i = jt + off - ro.base;
                if (i >= 0 && i < ro.n) ro.p[raw_pos(i)] = make_float2(z.x, z.y);
            }
            if constexpr (STORE) {
                if (OUT_MODE == OUT_REAL) OutIO<OutT>::store_real_one(p.out, jt + off, z.x);
                else OutIO<OutT>::store_one(p.out, jt + off, z.x, z.y);
            }
        }
    }

    // The last xs 16x16 sub-tiles of tile t alone, on the general path (the fused chain,
    // modem_chain.hip: the samples just before a workgroup's first tile, which its RX window
    // reads; the workgroup that owns tile t writes the same values there).
    __device__ __forceinline__ static void tail(const TxParams& p, _Float16* pl, const th4* lut_s, const th8 (&bh)[NKS],
                                const th8 (&bl)[NKS], int64_t t, int xs, cf2 unscale) {
        const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
        const int g0 = 4 * SUB - xs;                                // first sub-tile emitted
        stage_slow(p, pl, lut_s, t * TS - p.lead - PRE, g0 * 16 * SB);
        __syncthreads();
        const int64_t j0 = (t * TS - p.lead) * SPS;
#pragma unroll 1
        for (int q = 0; q < SUB; ++q) {
            if (wave * SUB + q < g0) continue;                      // wave-uniform
            f32x4 dre, dim;
            if (p.levels) fir<true>(pl, q, bh, bl, dre, dim);
            else fir<false>(pl, q, bh, bl, dre, dim);
            emit_edge(p, j0 + ((int64_t)(wave * SUB + q) * 16 * SB) * SPS, dre, dim, unscale);
        }
        __syncthreads();                                            // the planes are restaged next
    }

    // One tile t and, before it, the last xs sub-tiles of tile t - 1 (the fused small call,
    // modem_chain.hip: one RX tile per workgroup). The tail's symbol loads fly with the tile's
    // and the LUT's, both are staged before one barrier (the tail into the second plane set
    // pl2), and (RAW) every emitted sample is also written to the LDS window `ro`. The tail's
    // samples go to that window only: tile t - 1's workgroup stores them, and this workgroup's
    // RX reads its whole window from LDS, on the general path too (RxMfma::slow_tile<HO>).
    template <int BPS, bool RAW = true>
    __device__ __forceinline__ static void one_tile(const TxParams& p, _Float16* pl, _Float16* pl2, th4* lut_s,
                                                    const th8 (&bh)[NKS], const th8 (&bl)[NKS], int64_t t, int xs,
                                                    const RawOut& ro) {
        constexpr int NK = (NE + NT - 1) / NT;
        const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        const int kab = p.lut_scale_exp + p.tap_scale_exp;
        const float us = __builtin_ldexpf(1.0f, -kab);
        const cf2 unscale = {us, us};
        const int64_t ms = t * TS - p.lead - PRE, mlast = p.nsym_valid - 1;
        const bool fullt = BPS > 0 && ms >= 0 && ms + NE <= p.nsym_valid && t * TS - p.lead + TS <= p.nsym;
        Word<BPS> pre[U];
        if (fullt) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                int64_t m = ms + tid + NT * u;
                m = m < 0 ? 0 : (m > mlast ? mlast : m);
                pre[u] = load_word<BPS>(p.bits, m);
            }
        }
        const bool tl = xs > 0 && t > 0;
        const int g0 = 4 * SUB - xs, e_lo = g0 * 16 * SB;
        const int64_t ms2 = ms - TS;
        uint32_t idx[NK];
        float2 hv[NK];
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            const int e = tid + k * NT;
            const int64_t m = ms2 + e;
            idx[k] = 0;
            hv[k] = make_float2(0.f, 0.f);
            if (tl && e < NE && e >= e_lo) {
                if (m < 0) { if (m >= -(int64_t)(p.K - 1)) hv[k] = p.hist[m + p.K - 1]; }
                else if (m < p.nsym_valid) idx[k] = tx_symbol_index(p, m);
            }
        }
        const th4* lut_h = reinterpret_cast<const th4*>(p.lut_h);
        for (int i = tid; i < (1 << p.bps); i += NT) lut_s[i] = lut_h[i];
        __syncthreads();   // LUT visible
        if (fullt) {
            put_all<BPS>(pl, lut_s, pre);
        } else {
            stage_slow(p, pl, lut_s, ms);
        }
        if (tl) {
#pragma unroll
            for (int k = 0; k < NK; ++k) {
                const int e = tid + k * NT;
                const int64_t m = ms2 + e;
                if (e < NE && e >= e_lo) put(pl2, e, m >= 0 && m < p.nsym_valid ? lut_s[idx[k]] : split_value(p, hv[k]));
            }
        }
        __syncthreads();
        const int64_t j0 = (t * TS - p.lead) * SPS, j2 = j0 - (int64_t)TS * SPS;
        const bool lv = p.levels != 0;
#pragma unroll 1
        for (int q = 0; q < SUB; ++q) {
            const int g = wave * SUB + q;
            f32x4 dre, dim;
            if (tl && g >= g0) {                                    // wave-uniform
                if (lv) fir<true>(pl2, q, bh, bl, dre, dim);
                else fir<false>(pl2, q, bh, bl, dre, dim);
                emit_edge<RAW, !RAW>(p, j2 + ((int64_t)g * 16 * SB) * SPS, dre, dim, unscale, ro);
            }
            if (lv) fir<true>(pl, q, bh, bl, dre, dim);
            else fir<false>(pl, q, bh, bl, dre, dim);
            if (!RAW) __builtin_amdgcn_s_setprio(1);                // as run(): the epilogue issues first
            if (fullt) emit_full<RAW>(p, j0 + ((int64_t)g * 16 * SB) * SPS, dre, dim, unscale, ro);
            else emit_edge<RAW>(p, j0 + ((int64_t)g * 16 * SB) * SPS, dre, dim, unscale, ro);
            if (!RAW) __builtin_amdgcn_s_setprio(0);
        }
        __syncthreads();                                            // the planes are restaged next
    }

    // Tiles t0, t0 + ts, ... below t1 (xs > 0: first the last xs sub-tiles of tile t0 - 1). Tile t
    // holds symbols [t*TS - lead, (t+1)*TS - lead) of the call. BPS > 0: bits aligned, no leftover
    // bits, carrier index < 2^46 (the steady state); BPS == 0: general path only.
    template <int BPS>
    __device__ __forceinline__ static void run(const TxParams& p, _Float16* pl, th4* lut_s, const th8 (&bh)[NKS],
                               const th8 (&bl)[NKS], int64_t t0, int64_t t1, int64_t ts, int xs = 0) {
        const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        const int lead = p.lead;
        const int kab = p.lut_scale_exp + p.tap_scale_exp;
        const bool lv = p.levels != 0;
        const float us = __builtin_ldexpf(1.0f, -kab);             // exact (|kab| < 126)
        const cf2 unscale = {us, us};
        // full tile: every staged symbol is data of this call, every sample is emitted
        auto full = [&](int64_t t) {
            const int64_t ms = t * TS - lead - PRE;
            return BPS > 0 && ms >= 0 && ms + NE <= p.nsym_valid && t * TS - lead + TS <= p.nsym;
        };
        Word<BPS> pre[U];
        // tile t's bits words through a buffer descriptor from its window's first symbol (a full
        // tile's window lies inside the call; a prefetched tile that turns out not to be full is
        // staged by stage_slow instead, so the zeros its out-of-range words read are never used):
        // no per-slot 64-bit clamps (~35 VALU per tile and wave)
        auto prefetch = [&](int64_t t) {
            const int64_t ms = t * TS - lead - PRE;
            const int64_t mb = ms < 0 ? 0 : ms;
            const int64_t nrec = (p.nsym_valid - mb) * BPS;
            const __amdgpu_buffer_rsrc_t rb = buf_rsrc(p.bits + mb * BPS,
                                                       nrec <= 0 ? 0u : nrec > 0x7fffffff ? 0x7fffffffu : (uint32_t)nrec);
#pragma unroll
            for (int u = 0; u < U; ++u) pre[u] = load_word_rsrc<BPS>(rb, (tid + NT * u) * BPS);
        };
        int64_t t = t0;
        // the first tile's bits are requested before the LUT goes to LDS, so that the two
        // memory latencies at the kernel's start overlap
        bool ready = t < t1 && full(t);
        if (ready) prefetch(t);
        const th4* lut_h = reinterpret_cast<const th4*>(p.lut_h);
        for (int i = tid; i < (1 << p.bps); i += NT) lut_s[i] = lut_h[i];
        __syncthreads();   // LUT visible
        if (xs > 0 && t0 > 0) tail(p, pl, lut_s, bh, bl, t0 - 1, xs, unscale);
        while (t < t1) {
            if (full(t)) {
                if (!ready) prefetch(t);
                ready = false;
                // the first tile's bits complete before the loop: a load still pending on entry
                // merged into the loop head's wait tracking
#pragma unroll
                for (int u = 0; u < U; ++u) asm volatile("" ::"v"(pre[u]));
                // one full tile; NTT: its stores non-temporal (below tx_nt_below), a template
                // constant per loop so that no store sits under a runtime branch (emit_full)
                auto tile = [&](auto ntc) {
                    constexpr bool NTT = decltype(ntc)::value;
                    put_all<BPS>(pl, lut_s, pre);
                    __syncthreads();
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
                        emit_full<false, NTT>(p, j0 + ((int64_t)(wave * SUB + q) * 16 * SB) * SPS, dre, dim, unscale);
                        __builtin_amdgcn_s_setprio(0);
                    }
                    __syncthreads();                     // the window is restaged next trip
                };
                // tiles walk upwards: those wholly below tx_nt_below come first
                for (; t < t1 && full(t) && (t * TS - lead + TS) * SPS <= p.nt_below; t += ts) tile(std::true_type{});
                for (; t < t1 && full(t); t += ts) tile(std::false_type{});
            } else {
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
                t += ts;
            }
        }
    }
};

// This lane's B fragments (hi, lo) per k-step, from the host-built table. Each is pinned in its
// registers right here (an opaque asm use: the loads are waited for once, at the kernel's start):
// left pending, the compiler's wait tracking merged them into the tile loop's head and made the
// first MFMA of every tile wait for the next tile's bits prefetch (s_waitcnt vmcnt(3) of 5).
template <int NKS>
__device__ __forceinline__ void load_bfrag(const th8* __restrict__ bfrag, th8 (&bh)[NKS], th8 (&bl)[NKS]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
        bh[s] = bfrag[(2 * s) * 64 + lane];
        bl[s] = bfrag[(2 * s + 1) * 64 + lane];
    }
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
        asm volatile("" : "+v"(bh[s]));
        asm volatile("" : "+v"(bl[s]));
    }
}

// One channel's share of a launch: workgroup `bid` of `nb` working on channel p.
template <int SPS, int NKS, int OUT_MODE, typename OutT, int SUB>
__device__ __forceinline__ void tx_mfma_body(const TxParams& p, const th8* __restrict__ bfrag,
                                             int64_t bid, int64_t nb) {
    using K = TxMfma<SPS, NKS, OUT_MODE, OutT, SUB>;
    extern __shared__ __attribute__((aligned(16))) _Float16 lds_t[];
    _Float16* pl = lds_t;
    th4* lut_s = reinterpret_cast<th4*>(lds_t + K::PLANES);
    if (bid == 0) tx_state_update(p);
    th8 bh[NKS], bl[NKS];                        // this lane's B fragments (hi, lo) per k-step
    load_bfrag(bfrag, bh, bl);
    const int64_t ntiles = (p.nsym + p.lead + K::TS - 1) / K::TS;
    // tiles bid, bid + nb, ...: concurrently running workgroups work on neighbouring tiles
    // (measured 1 % faster on C3 than contiguous ranges per workgroup)
    const int64_t t0 = bid, t1 = ntiles, ts = nb;
    if (t0 >= t1) return;
    if (p.fast_bits && p.idx46 && K::out_ok(p)) {      // one uniform switch: the tile loop is specialised
        switch (p.bps) {
        case 1: K::template run<1>(p, pl, lut_s, bh, bl, t0, t1, ts); return;
        case 2: K::template run<2>(p, pl, lut_s, bh, bl, t0, t1, ts); return;
        case 4: K::template run<4>(p, pl, lut_s, bh, bl, t0, t1, ts); return;
        case 8: K::template run<8>(p, pl, lut_s, bh, bl, t0, t1, ts); return;
        }
    }
    K::template run<0>(p, pl, lut_s, bh, bl, t0, t1, ts);
}

// Tile size by the work: 4 sub-tiles per wave when the call has at least four such tiles
// per CU, else one (a small call, C2: 2^18 symbols, then still spreads over every SIMD). The
// 16x16 sub-tiles are computed alike either way: results do not depend on the choice.
inline bool tx_small_tiles(int64_t nsym, int sb) { return nsym < (int64_t)4 * 4 * 4 * 16 * sb * device_cus(); }

}  // namespace mk
