// rust-modem_amd/csrc/modem_rx_mfma.h — the RX matched filter on the matrix cores (RxMfma,
// rx_mfma_body) and the device helpers it shares with the other RX kernels: included by
// modem_rx.hip (rx_mfma, rx_mfma_batch) and modem_chain.hip (the fused TX->RX period).
#pragma once
#include "modem_device.h"
#include "libm_sincosf.h"

namespace mk {

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

// Real int16 samples (MODEM_DTYPE_I16, the `demodulate` reader): x = (v, 0).
template <> struct InIO<int16_t> {
    __device__ static float2 load(const void* x, int64_t q) {
        return make_float2((float)reinterpret_cast<const int16_t*>(x)[q], 0.f);
    }
    __device__ static void copy(void* dst, int64_t i, const void* src, int64_t q) {
        reinterpret_cast<int16_t*>(dst)[i] = reinterpret_cast<const int16_t*>(src)[q];
    }
};

enum { MIX_COMPLEX = 0, MIX_REFERENCE_REAL = 1, MIX_REFERENCE_REAL_EXACT = 2 };
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

// carrier.next() + pll.phase_offset (demodulator.rs:50): one f32 add, exact for offset 0
__device__ __forceinline__ float rx_phase(const RxParams& p, float carrier) {
#pragma clang fp contract(off)
    return carrier + p.phase_offset;
}

// sin / cos of carrier.next() + pll.phase_offset (demodulator.rs:50) on the hardware
// v_sin/v_cos (argument in turns): turns = fma(carrier, 1/2pi, offset/2pi), the same
// expression in every RX path (fast, general, VALU), so that results never depend on which
// path a sample took. For offset 0 it is fl(carrier / 2pi) exactly as __sinf/__cosf take it.
__device__ __forceinline__ void rx_sincos(const RxParams& p, float carrier, float& s, float& c) {
    const float rev = __builtin_fmaf(carrier, kRcp2Pi, p.phase_offset * kRcp2Pi);
    s = __builtin_amdgcn_sinf(rev);
    c = __builtin_amdgcn_cosf(rev);
}

// x * e^{-j phase} (or the reference's x.re * (cos, -sin), demodulator.rs:46,53-54) for
// stream index n = nb + off (nb wave-uniform).
template <int MIX>
__device__ __forceinline__ float2 rx_mix(const RxParams& p, int64_t nb, int off, float2 x) {
    if (nb + off < 0) return make_float2(0.f, 0.f);   // before the stream: zero history
    float s, c;
    rx_sincos(p, carrier_phase_off(p.w, p.c0 + (uint64_t)nb, off, p.exact_idx), s, c);
    if (MIX == MIX_REFERENCE_REAL) return make_float2(x.x * c, x.x * -s);
    return make_float2(__builtin_fmaf(x.y, s, x.x * c), __builtin_fmaf(-x.x, s, x.y * c));
}

// Nearest LUT entry, lowest index on ties (squared distance, no contraction).
__device__ __forceinline__ uint8_t rx_slice_nearest(const RxParams& p, float re, float im) {
#pragma clang fp contract(off)
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

// The same for a 4-entry LUT (QPSK), unrolled: the table stays in scalar registers across
// the tile loop instead of being re-read per decision.
__device__ __forceinline__ uint8_t rx_slice_nearest4(const RxParams& p, float re, float im) {
#pragma clang fp contract(off)
    cfloat* lut = (cfloat*)p.slut;
    uint32_t best = 0;
    float bd = __builtin_inff();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float dr = re - lut[2 * k], di = im - lut[2 * k + 1];
        const float d = dr * dr + di * di;
        if (d < bd) { bd = d; best = (uint32_t)k; }
    }
    return (uint8_t)best;
}

__device__ __forceinline__ uint8_t rx_slice(const RxParams& p, float re, float im) {
#pragma clang fp contract(off)
    if (p.slicer_kind == SLICER_QAM_AXIS) {
        const int ms = (int)p.max_symbol;
        const float fi = (re * p.inv_scale + p.max_symbol) * 0.5f;
        const float fq = (im * p.inv_scale + p.max_symbol) * 0.5f;
        const int si = (int)__builtin_fminf(__builtin_fmaxf(__builtin_rintf(fi), 0.f), p.max_symbol);
        const int sq = (int)__builtin_fminf(__builtin_fmaxf(__builtin_rintf(fq), 0.f), p.max_symbol);
        (void)ms;
        return (uint8_t)((si << p.bits_per_carrier) | sq);
    }
    return rx_slice_nearest(p, re, im);
}

template <typename OutT>
__device__ __forceinline__ void rx_emit(const RxParams& p, int64_t o, float re, float im) {
    if (p.out_iq) OutIO<OutT>::store_one(p.out_iq, o, re, im);
    if (p.out_sym && p.slicer_kind != SLICER_NONE) p.out_sym[o] = rx_slice(p, re, im);
}

template <typename InT>
__device__ inline void rx_state_update(const RxParams& p) {
    for (int i = threadIdx.x; i < p.HL; i += blockDim.x) {
        const int64_t q = p.N - p.HL + i;
        if (q >= 0) InIO<InT>::copy(p.hist_new, i, p.x, q);
        else InIO<InT>::copy(p.hist_new, i, p.hist, q + p.HL);
    }
}

// ----------------------------------------------------------------------- RX on MFMA ----
// Matched filter at the kept instants on the matrix cores (v_mfma_f32_16x16x32_f16):
//   rows i = 16 groups of 16 consecutive kept instants, cols c = instant in the group,
//   k = w = offset in a W = 32*NKS sample window ending at the group's last instant,
//   A[i][w] = z[start_i + w] (mixed input), B[w][c] = h[W - 1 - w - (15 - c)*DEC].
// Every real operand is split in two f16 halves, a = a_hi + a_lo (round to nearest), and
//   A*B ~= A_hi*B_hi + A_hi*B_lo + A_lo*B_hi      (dropped A_lo*B_lo < 2^-22 |a||b|)
// accumulates in f32: 6 MFMAs (re and im rails) per 32-sample k-step, 16x the MAC rate of
// the f32 MFMA. Range: the taps are scaled by 2^kb on the host (0 when their max is in
// [2^-3, 2^15)); the mixed samples of a tile by 2^ka, ka = tile_ka of the tile's max |z| (0
// inside [2^-3, 2^15), so results never depend on how a stream is cut into calls). Outputs
// are scaled back with ldexp (exact).
// LDS: four f16 planes (re_hi, re_lo, im_hi, im_lo) and NC shifted copies of the hi/lo
// reversed-tap table, so that every lane's 8-tap B read is one aligned ds_read_b128.

// Plane position of staged sample e: 16 pad halves after every RW samples. With the row pitch
// RW + 16 (= 2 mod 4 in 16-B units), the 16 lanes of each ds_read_b128 lane group (rows i at
// k-offset g, rows i' at g + 1) hit distinct bank quads; a pitch of RW + 8 was 2-way conflicted.
__host__ __device__ constexpr int rxh_pos(int e, int RW) { return e + 16 * (e / RW); }

// What the steady-state epilogue writes: baseband IQ, QAM-axis decisions, or both
// (RXE_GEN: any other combination, guarded per store).
enum { RXE_GEN = 0, RXE_IQ = 1, RXE_SYM = 2, RXE_IQSYM = 3, RXE_NEAREST = 4 };   // | NEAREST: LUT slicer

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// hi = rn_f16(v), lo = rn_f16(v - hi) for two values: one v_cvt_pk_f16_f32 and two
// v_fma_mix{lo,hi}_f16 that round the exact f32 remainder v - hi straight into the packed
// lo halves (3 VALU per pair).
__device__ __forceinline__ void split2(cf2 v, h2& hi, h2& lo) {
    hi = __builtin_convertvector(v, h2);
    uint32_t l;
    asm("v_fma_mixlo_f16 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=&v"(l) : "v"(hi), "v"(v.x));
    asm("v_fma_mixhi_f16 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(l) : "v"(hi), "v"(v.y));
    lo = __builtin_bit_cast(h2, l);
}

// Conjugate mix of one sample, packed: (re, im) = (x*cs + y*sn, y*cs - x*sn) with the same
// roundings as fma(y, sn, x*cs) / fma(-x, sn, y*cs). cssn = (cs, sn).
__device__ __forceinline__ cf2 cmix(cf2 x, cf2 cssn) {
    const cf2 t = x * cssn.xx;
    return __builtin_elementwise_fma(x.yx, (cf2){cssn.y, -cssn.y}, t);
}

// Four consecutive input samples (one lane's staging quad).
template <typename InT> struct Quad;
template <> struct Quad<float> {
    struct T { float4 a, b; };
    __device__ static void split(const T& t, float2 (&x)[4]) {
        x[0] = make_float2(t.a.x, t.a.y); x[1] = make_float2(t.a.z, t.a.w);
        x[2] = make_float2(t.b.x, t.b.y); x[3] = make_float2(t.b.z, t.b.w);
    }
};
template <> struct Quad<__half> {
    using T = uint4;
    __device__ static void split(const T& t, float2 (&x)[4]) {
        x[0] = __half22float2(*reinterpret_cast<const __half2*>(&t.x));
        x[1] = __half22float2(*reinterpret_cast<const __half2*>(&t.y));
        x[2] = __half22float2(*reinterpret_cast<const __half2*>(&t.z));
        x[3] = __half22float2(*reinterpret_cast<const __half2*>(&t.w));
    }
};

__device__ __forceinline__ float wave_max(float m) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = __builtin_fmaxf(m, __shfl_xor(m, off));
    return m;
}

// A tile's scale exponent ka as a function of the biased f32 exponent `ex` of its max |z|
// (the split-f16 window): 0 when the max lies in [2^-3, 2^15) (or is zero / subnormal /
// non-finite); otherwise the multiple of 8 that moves it into [2^-3, 2^5) (small tiles) or
// [2^7, 2^15) (large ones). A pure function of the tile's content, so the fast path (which
// stages with a predicted ka and keeps the tile only if the prediction equals this) and the
// general path give identical results; steps of 8 binades keep the prediction from the
// previous tile right for any slowly varying amplitude.
__device__ __forceinline__ int tile_ka(int ex) {
    if (ex <= 0 || ex >= 0xff || (ex >= 127 - 3 && ex < 127 + 15)) return 0;
    const int k = ex < 127 - 3 ? 8 * ((127 - 3 - ex + 7) / 8) : -8 * ((ex - (127 + 14) + 7) / 8);
    return k > 120 ? 120 : k;                                // 2^k stays a normal f32
}
__device__ __forceinline__ int f32_exp(float m) { return (int)((__float_as_uint(m) >> 23) & 0xff); }

// The tiles one workgroup runs, in order: first, first + step, ... (count of them), of the
// call's ntiles.
struct TileSeq { int64_t first, step, count, ntiles; };

// The fused small call's hand-off (RxMfma::run<EM, true>): the LDS copy of the samples the
// workgroup's TX emitted, call samples [base, base + n), and the value of *ka_in.
struct RxHandoff {
    const float2* raw;
    int64_t base;
    int n;
    int kin;
};

// clamp(v, 0, cap) of a wave-uniform 64-bit value with 32-bit scalar ops on its halves (a
// 64-bit compare would go through the vector unit: v_cmp_*_i64 from SGPR pairs).
__device__ __forceinline__ uint32_t clamp64_u32(int64_t v, uint32_t cap) {
    const int32_t hi = (int32_t)((uint64_t)v >> 32);
    const uint32_t lo = (uint32_t)(uint64_t)v;
    return hi < 0 ? 0u : hi > 0 ? cap : (lo < cap ? lo : cap);
}

// QAM-axis decisions for (re, im) at once (rx_slice's roundings, contract off), the scale and
// offset on the packed pipe.
__device__ __forceinline__ uint8_t rx_slice_qam2(const RxParams& p, float re, float im) {
#pragma clang fp contract(off)
    const cf2 f = ((cf2){re, im} * p.inv_scale + p.max_symbol) * 0.5f;
    const float ms = p.max_symbol;
    const int si = (int)__builtin_fminf(__builtin_fmaxf(__builtin_rintf(f.x), 0.f), ms);
    const int sq = (int)__builtin_fminf(__builtin_fmaxf(__builtin_rintf(f.y), 0.f), ms);
    return (uint8_t)((si << p.bits_per_carrier) | sq);
}

// One workgroup of 4 waves per tile of TS = 1024 kept instants (persistent: XCD-matched
// top-down rounds of tiles). Per tile the waves mix, scale and split the tile's input into the
// LDS planes, reloading every staging slot with the next tile's samples as soon as it is
// consumed (those loads are in flight through the rest of the staging, the matched filter
// and the stores), then run the matched filter (16 rows of 16 instants per wave) and store
// the outputs. Per staged sample the VALU does: the carrier index as one exact f32 add
// (idx_split), the bit-exact phase (phase_from_f2), the turns and v_sin/v_cos, the packed
// conjugate mix, an optional exact power-of-two scale, one v_max3 and the split.
//
// The f16 range: a tile is staged with a predicted tile_ka (the previous tile's; a call's
// first from where the previous call ended, a stream's first from its raw input) and each
// wave votes with three ballots whether the tile's max lies in that exponent's window. A tile
// outside it, and the call's first tile (its window reads the history), take the general
// path: per-sample loads, two passes, the same tile_ka -> identical results either way.
template <int DEC, int NKS, typename InT, int MIX, typename OutT, int NWF_ = 4, int KS_ = 1>
struct RxMfma {
    using Q = Quad<InT>;
    using QT = typename Q::T;
    // K-split (KS = 2): two waves per 16-row block, each summing half of its k-steps, the upper
    // wave's sums handed over in LDS; 8 waves stage and filter a tile, so a tile whose planes
    // leave room for only 2 workgroups per CU (C5 f32: 73 KB) still runs 4 waves per SIMD.
    static constexpr int KS = KS_;
    static constexpr int NT = 256 * KS;                         // 4 (KS = 2: 8) waves stage every tile
    static constexpr int NW = NT / 64;
    static constexpr int NWF = NWF_;                            // 16-row blocks per tile: 4, or 1 (small calls)
    static constexpr int TS = NWF * 256;                        // kept instants per tile
    static constexpr int RW = 16 * DEC;                         // samples per A row
    static constexpr int W = 32 * NKS;
    static constexpr int NS = (TS - 16) * DEC + W;              // samples staged per tile
    static constexpr int NQ = (NS + 3) / 4;                     // quads
    static constexpr int U = (NQ + NT - 1) / NT;                // quads per lane
    // 1024-instant tiles: the tile's last, partial slot holds NS - 4 NT (U - 1) <= NT samples
    // (C3: 128, C5: 512), staged one per lane (2 VGPRs for an f32 sample instead of a quad's 8:
    // the quad form spilled 16 bytes in C5's K-split kernel; at C3 the 6 VGPRs freed for the
    // matched filter took the RX 29.80 -> 29.54 us). UQ quads + that sample per lane.
    static constexpr bool P1 = NWF == 4 && NS - 4 * NT * (U - 1) <= NT;
    static constexpr int UQ = P1 ? U - 1 : U;
    using ST = typename std::conditional<std::is_same<InT, float>::value, float2, uint32_t>::type;
    // Plane layout. decim 4 and 8: unpadded, 16-B chunks XOR-swizzled within each row of
    // 8 (decim 4) or 16 (decim 8) chunks by the row bits — conflict-free A reads and staging
    // writes (tests/test_lds_banks.py) and no pad halves, which lets 4 workgroups share a CU
    // (decim 4; decim 8 with two planes). Otherwise rxh_pos.
    static constexpr bool SWZ = (DEC == 4 || DEC == 8) && (4 * NT) % 1024 == 0;
    __host__ __device__ static constexpr int ppos(int e) {
        return !SWZ ? rxh_pos(e, RW)
             : DEC == 4 ? ((((e >> 3) ^ (((e >> 7) & 3) << 1)) << 3) | (e & 7))
                        : ((((e >> 3) ^ (((e >> 7) & 7) << 1)) << 3) | (e & 7));
    }
    static constexpr int PL = SWZ ? (4 * NQ + 63) & ~63 : (rxh_pos(4 * NQ - 1, RW) + 1 + 7) & ~7;   // halves per plane
    // f16 samples in and out (the f16 storage sweep, SURVEY.md §8c tolerance 2^-10): the mixed
    // samples are staged as their f16 roundings only (two planes, re and im; the f32 path's
    // lo planes carry bits below the f16 output's precision: +2^-12.4 of max|y| before the
    // output rounding on C5, tests/test_gpu_range.py), 2 MFMAs per rail and k-step instead of
    // 3, and half the LDS: C5 f16 fits 4 workgroups per CU instead of 2. Otherwise four planes
    // (re_hi, re_lo, im_hi, im_lo).
    static constexpr bool HI = std::is_same<InT, __half>::value && std::is_same<OutT, __half>::value;
    static constexpr int NPL = HI ? 2 : 4;
    // The matched filter's summation order: for the configurations a K-split launch may run
    // (decim 8, >= 16 k-steps, four planes: C5 f32) every launch sums the first and the second
    // half of the k-steps separately and adds the two, whatever its KS, tile size or kernel
    // (single-side, chain), so that results still never depend on how a stream is cut into calls.
    static constexpr bool KSO = DEC == 8 && NKS >= 16 && NKS % 2 == 0 && !HI;
    static_assert(KS == 1 || (KS == 2 && KSO && NWF == 4), "K-split: C5-shaped f32 tiles only");
    static constexpr int NC = rx_mfma_table_copies(DEC);
    static constexpr int TB = rx_mfma_table_len(DEC, NKS);      // halves per table (hi or lo)
    // the planes, whose LDS the general path also uses for the raw window (NS float2, or NS
    // half2 for f16 input with HI: within NPL * PL halves either way), the tap tables, votes
    static constexpr int TBL_OFF = NPL * PL;                    // halves
    // + votes, maxima [NW each], and with KS = 2 the upper waves' partial sums (f32x4 re, im per
    // lane and block)
    static constexpr size_t PART_BYTES = KS > 1 ? (size_t)2 * NWF * 64 * 16 : 0;
    static constexpr size_t LDS_BYTES = (size_t)TBL_OFF * 2 + (size_t)NC * 2 * TB * 2 + 2 * NW * 4 + PART_BYTES;
    static constexpr int K_TAB8 = NC * 2 * TB / 8;              // 16-B chunks of the tap tables
    static constexpr float GAIN = MIX == MIX_REFERENCE_REAL ? 2.0f : 1.0f;
    // Waves per SIMD the registers are held to: 4 where the LDS lets 4 workgroups share a CU
    // (the matched filter then single-buffers its operands to fit 128 VGPRs), else the
    // compiler's choice.
    static constexpr int WPE = SWZ && (LDS_BYTES <= 40960 || KS == 2) ? 4 : 1;
    // WPE 4: the matched filter single-buffers its operands (one k-step's at a time) to fit 128
    // VGPRs; the other waves hide the LDS latency (double-buffered at 4 waves per SIMD, with the
    // last slots' reloads moved after the filter to free their registers: neutral on C3, slower
    // on C5 f16, profiles/r05_tx_wide.txt, r05_c2_floor_and_db.txt).
    static constexpr bool DBF = WPE < 4;
    static_assert((4 * NT) % RW == 0, "a staging slot spans whole rows");
    // plane offset between staging slots (the swizzle repeats every 1024 samples)
    static constexpr int SLOT_POS = SWZ ? 4 * NT : 4 * NT + 16 * (4 * NT / RW);

    // Rows hold 16 instants aligned to the absolute instant index (k % 16 == column), so an
    // instant's taps always fall at the same k positions of the 32-wide MFMA sums and the
    // result never depends on where a call starts. Tile t covers instants
    // k_first - lead + t*TS ..; outputs before k_first are computed and dropped.
    __device__ static int lead(const RxParams& p) { return (int)(p.k_first & 15); }
    __device__ static int64_t q_lo_of(const RxParams& p, int64_t t) {
        return (p.k_first - lead(p) + t * TS) * DEC + p.D + 15 * DEC - W + 1 - p.n_start;
    }

    // threadIdx.x as a value the compiler cannot hoist: every lane-dependent quantity is then
    // computed where it is used instead of once at the kernel entry, where kept live across
    // the tile loop it would spill (a kernel with scratch runs fewer waves per CU: 38 vs
    // 32.6 us on C3)
    __device__ static int tid_() {
        int t = threadIdx.x;
        asm volatile("" : "+v"(t));
        return t;
    }

    // Carrier index n_base + e as f32 for the staged samples e of a tile: n_base = A + b with A
    // a multiple of 2^s exactly representable in f32 (s from the tile's largest index) and b
    // < 2^22, so fl(A + (b + e)) — one f32 add of two exact values — is the correctly rounded
    // `n as f32` (needs every index < 2^46: RxParams::idx46, checked on the host).
    struct Idx { float a, bl; };
    __device__ static Idx idx_split(uint64_t n_base) {
        const uint64_t n_max = n_base + NS;
        const int e = 63 - __builtin_clzll(n_max | 1);
        const int sh = e > 23 ? e - 23 : 0;
        const uint64_t A = n_base & ~((1ull << sh) - 1);
        const float af = __builtin_ldexpf((float)(uint32_t)(A >> sh), sh);      // exact
        const uint32_t b = (uint32_t)(n_base - A) + 4u * (uint32_t)tid_();
        return Idx{__builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(uint32_t, af))),
                   (float)b};
    }

    // Window of a tile staged with exponent k (see tile_ka): [lo, hi) for its max |z|.
    __device__ static cf2 window(int k) {
        return k == 0 ? (cf2){0x1p-3f, 0x1p15f} : k > 0 ? (cf2){0x1p-3f, 0x1p5f} : (cf2){0x1p7f, 0x1p15f};
    }
    // After the barrier: do the waves' votes put the staged tile inside the window of k?
    // (k == 0 also accepts an all-zero / subnormal tile, whose tile_ka is 0.)
    __device__ static bool fast_ok(const int* votes, int k) {
        int f = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) f |= votes[w];
        const bool good = k == 0 ? !(f & 2) && ((f & 1) || !(f & 4)) : (f & 1) && !(f & 2);
        return __builtin_amdgcn_readfirstlane((int)good) != 0;
    }
    __device__ static int read_ka(const float* r) {
        float m = r[0];
#pragma unroll
        for (int w = 1; w < NW; ++w) m = __builtin_fmaxf(m, r[w]);
        return __builtin_amdgcn_readfirstlane(tile_ka(f32_exp(m)));
    }

    // Staging slot u of a tile through a buffer descriptor whose base is the tile window's
    // first sample and whose size is what of its 4 * NQ samples lies in the chunk (0 bytes: no
    // next tile). Loads past the size return zeros without touching memory (the spare lanes of
    // the last slot; a call's last tile; a workgroup's last tile), so the reload of every slot
    // is unconditional. The descriptor never reaches outside the call's buffer: only tiles whose
    // window starts inside the chunk take this path (Walk::nfull), and a window starting before
    // it (q_lo < 0, which a misclassified tile would have: round 5's forced-fast-path build read
    // before p.x and faulted) gets no records at all, so that its loads return zeros.
    __device__ static __amdgpu_buffer_rsrc_t window_rsrc(const RxParams& p, int64_t q_lo, bool live) {
        constexpr int S = sizeof(InT) * 2;
        const bool in = live && (int32_t)((uint64_t)q_lo >> 32) >= 0;     // q_lo >= 0, on 32-bit halves
        const int64_t qb = in ? q_lo : 0;
        const uint32_t w = clamp64_u32(p.N - qb, (uint32_t)(4 * NQ));
        return buf_rsrc(reinterpret_cast<const char*>(p.x) + qb * S, in ? w * (uint32_t)S : 0u);
    }
    // P1: lane tid's sample of the partial slot (window sample 4 NT (U - 1) + tid)
    __device__ static ST load_one(__amdgpu_buffer_rsrc_t r, int tid) {
        constexpr int S = sizeof(InT) * 2;
        const int o = (4 * NT * (U - 1) + tid) * S;
        if constexpr (std::is_same<InT, float>::value)
            return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(r, o, 0, 0));
        else
            return __builtin_amdgcn_raw_buffer_load_b32(r, o, 0, 0);
    }
    __device__ static float2 one_f2(const ST& v) {
        if constexpr (std::is_same<InT, float>::value) return v;
        else return __half22float2(__builtin_bit_cast(__half2, v));
    }
    __device__ static QT load_slot(__amdgpu_buffer_rsrc_t r, int voff, int u) {
        constexpr int S = sizeof(InT) * 2;
        const int o = voff + 4 * NT * u * S;
        if constexpr (std::is_same<InT, float>::value) {
            const f32x4 a = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, o, 0, 0));
            const f32x4 b = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, o + 16, 0, 0));
            return QT{make_float4(a[0], a[1], a[2], a[3]), make_float4(b[0], b[1], b[2], b[3])};
        } else {
            return __builtin_bit_cast(QT, __builtin_amdgcn_raw_buffer_load_b128(r, o, 0, 0));
        }
    }

    // One 16x16 output block per wave: rows 16 wave .. 16 wave + 15 of the tile. Lane
    // (i = lane & 15, g = lane >> 4) reads A row i, samples 32s + 8g .. +7, and
    // B[32s + 8g + j][c = i] = T[32s + 8g + j + (15 - c)*DEC] from the table copy that makes
    // the read aligned. WPE 4: one k-step's operands at a time (fewer registers; the other
    // waves hide the LDS latency); otherwise the next k-step's load during this one's MFMAs.
    // fir_part: k-steps [s0, s0 + NS_) of 16-row block blk, summed from zero.
    template <int NS_>
    __device__ static void fir_part(const _Float16* pl, const _Float16* tbl, int blk, int s0, f32x4& dre, f32x4& dim) {
        constexpr bool DB = DBF;
        const int lane = tid_() & 63;
        const int i = lane & 15, g = lane >> 4;
        const int ae = (16 * blk + i) * RW + 8 * g + 32 * s0;
        const int xb = 8 * g + (15 - i) * DEC;
        const int q = xb & 7;
        const _Float16* brow = tbl + (q / (8 / NC)) * 2 * TB + (xb - q) + 32 * s0;
        f32x4 r0 = {0.f, 0.f, 0.f, 0.f}, m0 = r0;
        h8 a[2][4], b[2][2];
        auto load = [&](int s, int c) {
            const _Float16* ap = pl + ppos(ae + 32 * s);
            a[c][0] = *reinterpret_cast<const h8*>(ap);
            if (HI) {
                a[c][2] = *reinterpret_cast<const h8*>(ap + PL);
            } else {
                a[c][1] = *reinterpret_cast<const h8*>(ap + PL);
                a[c][2] = *reinterpret_cast<const h8*>(ap + 2 * PL);
                a[c][3] = *reinterpret_cast<const h8*>(ap + 3 * PL);
            }
            b[c][0] = *reinterpret_cast<const h8*>(brow + 32 * s);
            b[c][1] = *reinterpret_cast<const h8*>(brow + TB + 32 * s);
        };
        if (DB) load(0, 0);
#pragma unroll
        for (int s = 0; s < NS_; ++s) {
            const int c = DB ? s & 1 : 0;
            if (!DB) load(s, 0);
            else if (s + 1 < NS_) load(s + 1, c ^ 1);
            r0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[c][0], b[c][0], r0, 0, 0, 0);
            m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[c][2], b[c][0], m0, 0, 0, 0);
            r0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[c][0], b[c][1], r0, 0, 0, 0);
            m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[c][2], b[c][1], m0, 0, 0, 0);
            if (!HI) {
                r0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[c][1], b[c][0], r0, 0, 0, 0);
                m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[c][3], b[c][0], m0, 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        dre = r0;
        dim = m0;
    }
    // The wave's whole block (KS = 1): KSO configurations as the two halves' sums added.
    __device__ static void fir(const _Float16* pl, const _Float16* tbl, f32x4& dre, f32x4& dim) {
        const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
        if constexpr (KSO) {
            f32x4 r1, m1;
            fir_part<NKS / 2>(pl, tbl, wave, 0, dre, dim);
            fir_part<NKS / 2>(pl, tbl, wave, NKS / 2, r1, m1);
            dre += r1;
            dim += m1;
        } else {
            fir_part<NKS>(pl, tbl, wave, 0, dre, dim);
        }
    }

    // The tile's matched filter and outputs (instants ot0 + 256 blk ..); returns with the planes
    // free for the next staging. KS = 1: waves < NWF filter their block, a barrier, then they store.
    // KS = 2: waves blk and blk + NWF each sum half of block blk's
    // k-steps (the same two halves fir adds); the upper wave hands its sums over in LDS before a
    // barrier, after which the planes may be restaged, and the lower wave adds them and stores.
    template <int EM>
    __device__ __forceinline__ static void filter_emit(const RxParams& p, const _Float16* pl, const _Float16* tbl,
                                                       f32x4* part, int64_t ot0, int kab) {
        const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
        f32x4 dre, dim;
        if constexpr (KS == 1) {
            const bool fw = NWF == NW || wave < NWF;   // uniform
            if (fw) fir(pl, tbl, dre, dim);
            // the planes are free once every wave has filtered: the outputs (slicer, stores) of
            // a wave that is done overlap the other waves' filters and the next tile's staging
            __syncthreads();
            if (fw) emit<EM>(p, ot0 + wave * 256, dre, dim, kab);
        } else {
            const int blk = wave % NWF, kh = wave / NWF;
            fir_part<NKS / 2>(pl, tbl, blk, kh * (NKS / 2), dre, dim);
            const int lane = tid_() & 63;
            f32x4* pr = part + 64 * blk + lane;               // [re | im][block][lane]: 16-B lane stride
            f32x4* pi = pr + 64 * NWF;
            if (kh == 1) { *pr = dre; *pi = dim; }
            __syncthreads();
            if (kh == 0) {
                dre += *pr;
                dim += *pi;
            }
            // every wave issues the stores, the upper ones past the call's last instant (their
            // descriptors hold no records: dropped), so that no store sits under a branch in the
            // tile loop (the compiler's wait tracking then lost count of them: each staging waited
            // for the previous tile's stores)
            // (the upper waves skip the LUT slicer's search: its decisions are dropped anyway)
            emit<EM>(p, kh == 0 ? ot0 + blk * 256 : p.nout, dre, dim, kab, kh != 0);
        }
    }

    // Split z (4 samples) and write it at plane offset o (HI: the f16 roundings only).
    __device__ static void put4(_Float16* pl, int o, const float (&zr)[4], const float (&zi)[4]) {
        if constexpr (HI) {
            const h2 r0 = __builtin_convertvector((cf2){zr[0], zr[1]}, h2), r1 = __builtin_convertvector((cf2){zr[2], zr[3]}, h2);
            const h2 i0 = __builtin_convertvector((cf2){zi[0], zi[1]}, h2), i1 = __builtin_convertvector((cf2){zi[2], zi[3]}, h2);
            *reinterpret_cast<h4*>(pl + o) = (h4){r0.x, r0.y, r1.x, r1.y};
            *reinterpret_cast<h4*>(pl + PL + o) = (h4){i0.x, i0.y, i1.x, i1.y};
            return;
        }
        h2 rh0, rl0, rh1, rl1, ih0, il0, ih1, il1;
        split2((cf2){zr[0], zr[1]}, rh0, rl0);
        split2((cf2){zr[2], zr[3]}, rh1, rl1);
        split2((cf2){zi[0], zi[1]}, ih0, il0);
        split2((cf2){zi[2], zi[3]}, ih1, il1);
        *reinterpret_cast<h4*>(pl + o) = (h4){rh0.x, rh0.y, rh1.x, rh1.y};
        *reinterpret_cast<h4*>(pl + PL + o) = (h4){rl0.x, rl0.y, rl1.x, rl1.y};
        *reinterpret_cast<h4*>(pl + 2 * PL + o) = (h4){ih0.x, ih0.y, ih1.x, ih1.y};
        *reinterpret_cast<h4*>(pl + 3 * PL + o) = (h4){il0.x, il0.y, il1.x, il1.y};
    }

    // Fast-path staging of one tile from the prefetched registers `pre` at scale 2^k (SC:
    // k != 0; sc = 2^k, win = window(k)), reloading each slot with the next tile's samples
    // (`nxt`). Each wave writes its three votes (max >= window lo, >= window hi, normal).
    template <bool SC>
    __device__ static void stage(const RxParams& p, _Float16* pl, int* vote, Idx ix, float sc, cf2 win,
                                 QT (&pre)[UQ], ST& ps, __amdgpu_buffer_rsrc_t nxt) {
        const int tid = tid_();
        int pos0 = ppos(4 * tid);
        int voff = 4 * tid * (int)sizeof(InT) * 2;
        float bl = ix.bl;
        asm volatile("" : "+v"(pos0), "+v"(voff), "+v"(bl));
        const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        const float roff = p.phase_offset * kRcp2Pi;          // rx_sincos: carrier + PLL offset, in turns
        float mx = 0.f;
#pragma unroll
        for (int u = 0; u < UQ; ++u) {
            if ((u + 1) * NT > NQ && 64 * wave + NT * u >= NQ) {   // partial last slot: not this wave's
                pre[u] = load_slot(nxt, voff, u);
                continue;
            }
            float2 x[4];
            Q::split(pre[u], x);
            const int e0 = 4 * (tid + NT * u);
            const float bu = bl + (float)(4 * NT * u);
            const cf4 nf = (bu + (cf4){0.f, 1.f, 2.f, 3.f}) + ix.a;   // exact, then one rounding
            const cf4 rv = __builtin_elementwise_fma(phase_from_f4(p.w, nf), (cf4){kRcp2Pi, kRcp2Pi, kRcp2Pi, kRcp2Pi},
                                                     (cf4){roff, roff, roff, roff});
            const float sn[4] = {__builtin_amdgcn_sinf(rv.x), __builtin_amdgcn_sinf(rv.y),
                                 __builtin_amdgcn_sinf(rv.z), __builtin_amdgcn_sinf(rv.w)};
            const float cs[4] = {__builtin_amdgcn_cosf(rv.x), __builtin_amdgcn_cosf(rv.y),
                                 __builtin_amdgcn_cosf(rv.z), __builtin_amdgcn_cosf(rv.w)};
            float zr[4], zi[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                cf2 z = MIX == MIX_REFERENCE_REAL ? (cf2){x[j].x * cs[j], x[j].x * -sn[j]}
                                                  : cmix((cf2){x[j].x, x[j].y}, (cf2){cs[j], sn[j]});
                if (SC) z = z * sc;
                zr[j] = z.x;
                zi[j] = z.y;
                // only the last slot can reach past the tile: its extra samples are not counted
                if ((u + 1) * 4 * NT <= NS || e0 + j < NS)
                    asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(mx) : "v"(zr[j]), "v"(zi[j]));
            }
            if ((u + 1) * 4 * NT <= NS || e0 < NS) put4(pl, pos0 + u * SLOT_POS, zr, zi);
            // (not hoisted above the mix: the slot's registers would be copied out first)
            __builtin_amdgcn_sched_barrier(0);
            pre[u] = load_slot(nxt, voff, u);   // the next tile's slot u, same registers
            __builtin_amdgcn_sched_barrier(0);                 // one quad's temporaries at a time
        }
        if constexpr (P1) {                    // the partial slot, one sample per lane: the quad path's
            const int e = 4 * NT * (U - 1) + tid;               // arithmetic for sample e, bit for bit
            if (e < NS) {
                const float2 x = one_f2(ps);
                const float nf = (bl + (float)(4 * NT * (U - 1) - 3 * tid)) + ix.a;   // (b + e) exact, one rounding
                const float rv = __builtin_fmaf(phase_from_f2(p.w, (cf2){nf, nf}).x, kRcp2Pi, roff);
                const float sn = __builtin_amdgcn_sinf(rv), cs = __builtin_amdgcn_cosf(rv);
                cf2 z = MIX == MIX_REFERENCE_REAL ? (cf2){x.x * cs, x.x * -sn} : cmix((cf2){x.x, x.y}, (cf2){cs, sn});
                if (SC) z = z * sc;
                asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(mx) : "v"(z.x), "v"(z.y));
                const int o = ppos(e);
                if constexpr (HI) {            // two planes, the f16 roundings only (as put4)
                    const h2 h = __builtin_convertvector(z, h2);
                    pl[o] = h.x;
                    pl[PL + o] = h.y;
                } else {
                    h2 hi, lo;
                    split2(z, hi, lo);
                    pl[o] = hi.x;
                    pl[PL + o] = lo.x;
                    pl[2 * PL + o] = hi.y;
                    pl[3 * PL + o] = lo.y;
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            ps = load_one(nxt, tid);
        }
        // three votes per wave instead of a max reduction
        const bool blo = __ballot(mx >= win.x) != 0, bhi = __ballot(mx >= win.y) != 0,
                   bn = __ballot(mx >= 0x1p-126f) != 0;
        if ((tid & 63) == 0) vote[wave] = (blo ? 1 : 0) | (bhi ? 2 : 0) | (bn ? 4 : 0);
    }

    // D[row][col]: row = 4*(lane>>4) + r, col = lane&15 -> instant ot + 16*row + col. Stores
    // through buffer descriptors over the wave's instants that are in the call: those before
    // the call's first (ot < 0: a lane offset below the base wraps out of range) and past its
    // last are dropped without a branch.
    // dead (wave-uniform): every store of the wave lies past the call (the K-split's upper waves),
    // so the LUT slicer's search is skipped; the stores themselves stay unconditional.
    template <int EM>
    __device__ static void emit(const RxParams& p, int64_t ot, const f32x4& dre, const f32x4& dim, int kab,
                                bool dead = false) {
        const int lane = tid_() & 63;
        if (EM == RXE_GEN) {                   // any other output combination: guarded stores
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t o = ot + 16 * (4 * (lane >> 4) + r) + (lane & 15);
                if (o >= 0 && o < p.nout)
                    rx_emit<OutT>(p, o, GAIN * __builtin_ldexpf(dre[r], -kab), GAIN * __builtin_ldexpf(dim[r], -kab));
            }
            return;
        }
        const bool neg = (int32_t)((uint64_t)ot >> 32) < 0;   // before the call's first instant
        const int64_t ob = neg ? 0 : ot;
        const int sh = neg ? (int)ot : 0;                    // -15 .. 0
        const uint32_t nk = clamp64_u32(p.nout - ob, 256u);
        const __amdgpu_buffer_rsrc_t riq = buf_rsrc(reinterpret_cast<OutT*>(p.out_iq) + 2 * ob, nk * 2 * sizeof(OutT));
        const __amdgpu_buffer_rsrc_t rsy = buf_rsrc(p.out_sym + ob, nk);
        f32x4 re = dre, im = dim;
        if (kab != 0) {                        // uniform
#pragma unroll
            for (int r = 0; r < 4; ++r) { re[r] = __builtin_ldexpf(re[r], -kab); im[r] = __builtin_ldexpf(im[r], -kab); }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t off = (uint32_t)(16 * (4 * (lane >> 4) + r) + (lane & 15) + sh);
            const float a = re[r] * GAIN, b = im[r] * GAIN;
            if (EM & RXE_IQ) {
                if constexpr (std::is_same<OutT, float>::value)
                    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, make_float2(a, b)), riq, 8 * off, 0, 0);
                else
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, __floats2half2_rn(a, b)), riq, 4 * off, 0, 0);
            }
            if (EM & RXE_SYM) {
                const uint8_t sy = !(EM & RXE_NEAREST) ? rx_slice_qam2(p, a, b)
                                 : dead ? (uint8_t)0
                                 : p.bps == 2 ? rx_slice_nearest4(p, a, b) : rx_slice_nearest(p, a, b);
                __builtin_amdgcn_raw_buffer_store_b8(sy, rsy, off, 0, 0);
            }
        }
    }

    // General path for tile t (all waves): two passes over its samples (max, then tile_ka
    // scale + split), the matched filter, the outputs in range. Returns its tile_ka.
    // HO (the fused small call): the window's samples of the call come from the LDS copy of
    // what this workgroup's TX emitted (ho), not from HBM (the tail sub-tiles are only there).
    template <int EM, bool HO = false>
    __device__ __forceinline__ static int slow_tile(const RxParams& p, _Float16* pl, const _Float16* tbl, float* reds, f32x4* part,
                                    int64_t t, int kb, int ld, const RxHandoff& ho = RxHandoff{}) {
        // lane values recomputed here, not hoisted to the kernel entry (where, live across
        // the tile loop, they would spill)
        const int tid = tid_();
        const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        const int64_t q_lo = q_lo_of(p, t), n_lo = q_lo + p.n_start;
        // 1. The window's raw samples into the planes' LDS (free until this tile is staged),
        //    through a buffer descriptor over the chunk (out of range loads return zeros without
        //    a memory access, so they carry no branches), issued in batches of 8 per lane with
        //    the LDS writes after each batch: the compiler otherwise waited for every load pair
        //    before issuing the next (vmcnt(0) per sample), 17 round trips on C3 — the call's
        //    first tile took 10-16 us against ~3.5 for a fast one (r03 stamps, tools/stamps.py).
        //    The window's samples before the chunk (only a call's first tile has them) are then
        //    patched in from the history.
        // raw window: float2, or the exact half2 inputs when HI (it must fit the two planes)
        using RawT = typename std::conditional<HI, __half2, float2>::type;
        RawT* raw = reinterpret_cast<RawT*>(pl);
        static_assert((size_t)NS * sizeof(RawT) <= (size_t)NPL * PL * 2, "raw window within the planes' LDS");
        {
            constexpr int S = sizeof(InT) * 2;
            constexpr int NK = (NS + NT - 1) / NT, BATCH = 8;
            const int64_t ex = q_lo >= 0 ? 0 : -q_lo;                 // first window sample in the chunk
            const int64_t qx = q_lo + ex;
            const int64_t nx = p.N - qx < NS ? p.N - qx : NS;
            const __amdgpu_buffer_rsrc_t rx = buf_rsrc(reinterpret_cast<const char*>(p.x) + qx * S,
                                                       (uint32_t)(nx > 0 ? nx : 0) * S);
            const int ox = (int)ex;
            auto ld = [&](__amdgpu_buffer_rsrc_t r, uint32_t off) -> RawT {
                if constexpr (std::is_same<InT, float>::value)
                    return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
                else if constexpr (HI)
                    return __builtin_bit_cast(__half2, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
                else
                    return __half22float2(__builtin_bit_cast(__half2, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0)));
            };
#pragma unroll
            for (int k0 = 0; k0 < NK; k0 += BATCH) {
                RawT v[BATCH];
#pragma unroll
                for (int b = 0; b < BATCH; ++b) {     // < 0: wraps, out of range -> 0
                    if (k0 + b >= NK) continue;
                    if constexpr (HO) {                // (samples before the chunk: patched below)
                        const int64_t i = q_lo + (tid + (k0 + b) * NT) - ho.base;
                        const bool in = i >= 0 && i < ho.n && q_lo + (tid + (k0 + b) * NT) < p.N;
                        v[b] = in ? ho.raw[raw_pos(i)] : make_float2(0.f, 0.f);
                    } else {
                        v[b] = ld(rx, (uint32_t)(tid + (k0 + b) * NT - ox) * S);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int b = 0; b < BATCH; ++b) {
                    const int e = tid + (k0 + b) * NT;
                    if (k0 + b < NK && ((k0 + b + 1) * NT <= NS || e < NS)) raw[e] = v[b];
                }
            }
            if (ox > 0) {                                             // uniform: the call's first tile
                const int64_t hb = q_lo + p.HL;                       // history index of sample 0
                const int64_t eh = hb >= 0 ? 0 : -hb;                 // first window sample in the history
                const int64_t nhist = p.HL - (hb + eh);
                const __amdgpu_buffer_rsrc_t rh = buf_rsrc(reinterpret_cast<const char*>(p.hist) + (hb + eh) * S,
                                                           (uint32_t)(nhist > 0 ? nhist : 0) * S);
                const int oh = (int)eh;
                for (int k = 0; k * NT < ox && k < NK; ++k) {         // uniform bounds
                    const int e = tid + k * NT;
                    const RawT w = ld(rh, (uint32_t)(e - oh) * S);
                    if (e < ox && e < NS) raw[e] = w;
                }
            }
        }
        __syncthreads();
        // 2. Mix (rx_mix: the same values as the fast path's), the tile's max.
        float zr[U][4], zi[U][4];
        float mx = 0.f;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e0 = 4 * (tid + NT * u);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float2 z = make_float2(0.f, 0.f);
                if (e0 + j < NS) {
                    if constexpr (HI) z = rx_mix<MIX>(p, n_lo, e0 + j, __half22float2(raw[e0 + j]));
                    else z = rx_mix<MIX>(p, n_lo, e0 + j, raw[e0 + j]);
                }
                zr[u][j] = z.x;
                zi[u][j] = z.y;
                mx = __builtin_fmaxf(mx, __builtin_fmaxf(__builtin_fabsf(z.x), __builtin_fabsf(z.y)));
            }
        }
        mx = wave_max(mx);
        if ((tid & 63) == 0) reds[wave] = mx;
        __syncthreads();                       // also: every raw read done before the planes overwrite it
        // 3. Scale by 2^tile_ka, split, stage.
        const int ka = read_ka(reds);
        const float sc = __builtin_ldexpf(1.0f, ka);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e0 = 4 * (tid + NT * u);
            if (e0 >= NS) continue;
            float a[4], b[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) { a[j] = zr[u][j] * sc; b[j] = zi[u][j] * sc; }
            put4(pl, ppos(e0), a, b);
        }
        __syncthreads();
        filter_emit<EM>(p, pl, tbl, part, t * TS - ld, ka + kb);   // ends with the planes free
        return ka;
    }

    // A tile on the fast path: its window starts inside the chunk and its first instant is
    // kept (samples past the chunk's end load as zeros and instants past the call's last are
    // not stored, both through the buffer descriptors' bounds); the call's first tile, which
    // reads the history, takes the general path. `fast`: 4-B aligned input, carrier indices
    // < 2^46 (idx_split).
    struct Ctx {
        bool fast;
        int kb, ld;
    };

    // The workgroup's tiles t_i = first + i * step (i < count, step = -grid: top-down), walked
    // with running values so that a tile's scalar bookkeeping is a few adds, not 64-bit
    // multiplies and compares (100 extra s_nop per tile cost the RX 0.4-0.7 us,
    // profiles/r03_sensitivity.txt): the tile, its window offset q = q_lo_of(t), and the
    // number of leading tiles on the fast path (q and t only decrease along the walk, so the
    // tiles with q >= 0 and t * TS >= lead come first).
    struct Walk {
        int64_t t, q, step, dq, last;          // tile, q_lo_of(t), steps per tile, the call's last tile
        int32_t i, count, nfull;               // position, tiles in the walk, leading full tiles
        __device__ void next() { ++i; t += step; q += dq; }
        __device__ bool full() const { return i < nfull; }
        __device__ bool next_full() const { return i + 1 < nfull && i + 1 < count; }
    };
    __device__ static Walk walk(const RxParams& p, const TileSeq& sq, bool fast) {
        Walk w;
        w.t = sq.first;
        w.step = sq.step;
        w.dq = sq.step * (int64_t)(TS * DEC);
        w.q = q_lo_of(p, sq.first);
        w.last = sq.ntiles - 1;
        w.i = 0;
        w.count = (int32_t)sq.count;
        w.nfull = 0;
        if (fast) {                            // the smallest full tile: q_lo_of(t) >= 0, t * TS >= lead
            const int64_t q0 = q_lo_of(p, 0);
            int64_t tmin = q0 >= 0 ? 0 : (-q0 + TS * DEC - 1) / (TS * DEC);
            if (lead(p) > 0 && tmin < 1) tmin = 1;
            if (sq.first >= tmin) {
                const int64_t n = (sq.first - tmin) / -sq.step + 1;
                w.nfull = (int32_t)(n < sq.count ? n : sq.count);
            }
        }
        return w;
    }

    // Tiles from w.i on while their staging exponent keeps its class (SC: nonzero). Returns
    // at the end of the walk, or after the barrier of a tile the general path must redo.
    template <bool SC, int EM>
    __device__ __forceinline__ static void loop(const RxParams& p, _Float16* pl, const _Float16* tbl, int* votes, f32x4* part,
                                Walk& w, const Ctx& cx, QT (&pre)[UQ], ST& ps, int kpred) {
        const float sc = __builtin_ldexpf(1.0f, kpred);
        const cf2 win = window(kpred);
        bool last = false;
        __amdgpu_buffer_rsrc_t nxt;
        // stage the tile at w.i (reloading the registers with the next tile's window) and check its
        // votes: false = the general path redoes it. Called before the loop and at the end of its
        // body, so that every path into the loop head has issued the staging's reloads last: with
        // the staging at the head, the vote's exit and the loop's latch shared a block, and the
        // compiler's wait tracking, merging a path without the tile's I/Q and decision stores,
        // made each staging wait for the previous tile's stores to complete.
        auto stage_tile = [&]() -> bool {
            const bool fi = w.full();
            const bool pf = w.next_full();
            nxt = window_rsrc(p, pf ? w.q + w.dq : 0, pf);
            const Idx ix = idx_split(p.c0 + (uint64_t)(w.q + p.n_start));
            // the staging (VALU-bound, the limiting stage) issues ahead of the other
            // workgroups' filter and stores on the SIMD: C3 RX 31.6-31.8 -> 31.0-31.4 us by
            // event, +0.8 % bench (profiles/r02_store_layout_ab.txt; priority 3: no better)
            __builtin_amdgcn_s_setprio(1);
            stage<SC>(p, pl, votes, ix, sc, win, pre, ps, nxt);
            __builtin_amdgcn_s_setprio(0);
            __syncthreads();
            return fi && fast_ok(votes, kpred);
        };
        if (w.i >= w.count || !stage_tile()) return;
        for (;;) {
            const int64_t t = w.t;
            last |= t == w.last;
            filter_emit<EM>(p, pl, tbl, part, t * TS - cx.ld, kpred + cx.kb);   // planes free after it
            w.next();
            if (w.i >= w.count || !stage_tile()) break;
        }
        // the call's last tile: its exponent is where the next call's prediction starts (stored
        // after the loop: a store under a branch in it would break the wait tracking likewise)
        if (last && threadIdx.x == 0) *p.ka_out = kpred;
    }

    // HO (the fused small call, modem_chain.hip): the tap tables are already in LDS, `ho.kin`
    // holds *p.ka_in, and the tile reads its window from the LDS copy of the samples this
    // workgroup's TX emitted (ho.raw) instead of from HBM, on the fast and the general path
    // (samples before the call from the history, as always).
    template <int EM, bool HO = false>
    __device__ __forceinline__ static void run(const RxParams& p, _Float16* pl, _Float16* tbl, const _Float16* __restrict__ tables,
                               float* red, const TileSeq sq, int64_t bid, const RxHandoff& ho = RxHandoff{}) {
        const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
        const Ctx cx{p.idx46 && ((uintptr_t)p.x & 3) == 0, p.tap_scale_exp, lead(p)};
        Walk w = walk(p, sq, cx.fast);
        int* votes = reinterpret_cast<int*>(red);            // [NW]
        float* reds = red + NW;                              // [NW]
        f32x4* part = reinterpret_cast<f32x4*>(red + 2 * NW);   // KS = 2: [2][NWF][64]
        QT pre[UQ];
        ST ps{};                                             // P1: the partial slot's sample
        auto prefetch = [&](int64_t q, bool live) {
            const __amdgpu_buffer_rsrc_t r = window_rsrc(p, live ? q : 0, live);
            const int voff = 4 * tid_() * (int)sizeof(InT) * 2;
#pragma unroll
            for (int u = 0; u < UQ; ++u) pre[u] = load_slot(r, voff, u);
            if constexpr (P1) ps = load_one(r, tid_());
        };
        // the tap tables into LDS, their loads issued before the first tile's so that the two
        // memory latencies at the kernel's start overlap (the table stores wait for the table
        // loads only)
        constexpr int NTB = K_TAB8 / NT + (K_TAB8 % NT ? 1 : 0);
        const bool f0 = w.full();
        if constexpr (HO) {
            static_assert(std::is_same<InT, float>::value, "LDS hand-off: f32 samples");
            static_assert(!P1, "LDS hand-off: quad slots");
            if (!f0) {
#pragma unroll
                for (int u = 0; u < UQ; ++u) pre[u] = QT{make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
            } else {                           // the window from the LDS copy (zeros past it and the call)
                const int e = 4 * tid_();
#pragma unroll
                for (int u = 0; u < UQ; ++u) {
                    float2 x[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int eu = e + 4 * NT * u + j;
                        const int64_t i = w.q + eu - ho.base;
                        x[j] = eu < 4 * NQ && w.q + eu < p.N && i >= 0 && i < ho.n ? ho.raw[raw_pos(i)] : make_float2(0.f, 0.f);
                    }
                    pre[u] = QT{make_float4(x[0].x, x[0].y, x[1].x, x[1].y), make_float4(x[2].x, x[2].y, x[3].x, x[3].y)};
                }
            }
        } else {
            h8 tv[NTB];
#pragma unroll
            for (int k = 0; k < NTB; ++k) {
                const int j = tid_() + k * NT;
                if (j < K_TAB8) tv[k] = reinterpret_cast<const h8*>(tables)[j];
            }
            prefetch(w.q, f0);
#pragma unroll
            for (int k = 0; k < NTB; ++k) {
                const int j = tid_() + k * NT;
                if (j < K_TAB8) reinterpret_cast<h8*>(tbl)[j] = tv[k];
            }
        }
        __syncthreads();
        // the first prediction: where the previous call ended (any exponent tile_ka can give)
        const int kin = HO ? ho.kin : *p.ka_in;
        int kpred = kin >= -120 && kin <= 120 && (kin & 7) == 0 ? kin : 0;
        if (f0 && kin == INT32_MIN) {          // a stream's first call: from the first tile's raw input
            float mx = 0.f;
            if constexpr (P1) {                // (zeros past the window)
                const float2 x = one_f2(ps);
                asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(mx) : "v"(x.x), "v"(x.y));
            }
#pragma unroll
            for (int u = 0; u < UQ; ++u) {
                if ((u + 1) * NT > NQ && 64 * wave + NT * u >= NQ) continue;
                float2 x[4];
                Q::split(pre[u], x);
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(mx) : "v"(x[j].x), "v"(x[j].y));
            }
            mx = wave_max(mx);
            if ((tid_() & 63) == 0) reds[wave] = mx;
            __syncthreads();
            kpred = read_ka(reds);
            __syncthreads();
        }
        while (w.i < w.count) {
            if (kpred == 0) loop<false, EM>(p, pl, tbl, votes, part, w, cx, pre, ps, kpred);
            else loop<true, EM>(p, pl, tbl, votes, part, w, cx, pre, ps, kpred);
            if (w.i < w.count) {               // tile w.t on the general path (one place in the code)
                kpred = slow_tile<EM, HO>(p, pl, tbl, reds, part, w.t, cx.kb, cx.ld, ho);
                if (w.t == w.last && threadIdx.x == 0) *p.ka_out = kpred;   // the call's last tile
                w.next();
                // reload the next tile (what the staging of tile i loaded is dropped: `pre` is
                // not held across the general path, which has no registers to spare)
                prefetch(w.q, w.i < w.count && w.full());
            }
        }
    }
};

// One channel's share of a launch: workgroup `bid` of `nb` working on channel p, with the
// epilogue EM chosen on the host (rx_mfma_em): each kernel keeps only its own stores.
template <int DEC, int NKS, typename InT, int MIX, typename OutT, int NWF, int EM, int KS = 1>
__device__ __forceinline__ void rx_mfma_body(const RxParams& p, const _Float16* __restrict__ tables, int64_t bid,
                                             int64_t nb) {
    using K = RxMfma<DEC, NKS, InT, MIX, OutT, NWF, KS>;
    extern __shared__ __attribute__((aligned(16))) _Float16 lds_h[];
    _Float16* pl = lds_h;                                   // 4 sample planes
    _Float16* tbl = lds_h + K::TBL_OFF;                     // NC x (hi, lo) tap tables
    float* red = reinterpret_cast<float*>(tbl + K::NC * 2 * K::TB);
    if (bid == 0) rx_state_update<InT>(p);
    const int64_t ntiles = (p.nout + K::lead(p) + K::TS - 1) / K::TS;
    // Rounds of nb tiles from the top down, tile R - (r + 1) nb + bid in round r. The TX hands
    // its tiles out grid-strided (tile i to workgroup i mod grid, both grids multiples of 8, so
    // tile i is written on XCD slot i mod 8); the RX's first round then reads the ~32 MiB the
    // TX wrote last, each tile on the XCD slot that wrote it (blocks b and b + 8 share an XCD).
    // C3: 35.0 -> 33.8 us against contiguous ranges per workgroup; the same rounds with the
    // slots shifted by 1 or 4 measured 38.1-39.1 us (PMC FETCH_SIZE per launch unchanged).
    if (ntiles <= 0) {                         // no tile: the next call predicts as this one did
        if (bid == 0 && threadIdx.x == 0) *p.ka_out = *p.ka_in;
        return;
    }
    static_assert(kRxTilesTopDown, "the TX store policy (tx_nt_below) assumes the top-down walk");
    const int64_t R = (ntiles + nb - 1) / nb * nb;
    TileSeq sq{R - nb + bid, -nb, R / nb, ntiles};
    if (sq.first >= ntiles) { sq.first -= nb; --sq.count; }
    if (sq.count <= 0) return;
    K::template run<EM>(p, pl, tbl, tables, red, sq, bid);
}

// The epilogue specialisation for a call: stores known at compile time for the loopback
// chain's outputs (f32 or f16 I/Q in and out, complex mix), else the guarded general one.
template <typename InT, int MIX, typename OutT>
__host__ inline int rx_mfma_em(const RxParams& p) {
    const bool loop = std::is_same<InT, OutT>::value && MIX == MIX_COMPLEX;
    if (!loop) return RXE_GEN;
    const bool qam = p.slicer_kind == SLICER_QAM_AXIS && p.out_sym;
    if (p.out_iq && qam) return RXE_IQSYM;
    if (std::is_same<InT, float>::value) {
        if (p.out_iq && p.out_sym && p.slicer_kind == SLICER_NEAREST) return RXE_IQSYM | RXE_NEAREST;
        if (p.out_iq && !p.out_sym) return RXE_IQ;
        if (!p.out_iq && qam) return RXE_SYM;
    }
    return RXE_GEN;
}

// Tile size by the work: 1024-instant tiles (4 filter waves) when the call has at least four
// per CU, else 256-instant tiles staged by 4 waves and filtered by one, so that a small call
// (C2: 2^18 instants) still spreads its staging over every SIMD. The filter of a 16-instant
// row is the same code either way: results do not depend on the choice.
inline bool rx_small_tiles(int64_t ninst) { return ninst < (int64_t)4 * 1024 * device_cus(); }

}  // namespace mk
