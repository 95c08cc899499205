// rust-modem_amd/csrc/modem_rx.hip — gfx950 RX kernels (demodulator.rs:44-56 + fir.rs:18-34,
// evaluated only at the kept instants): mix -> matched filter -> decimate -> slicer.
// RX  (demodulator.rs:44-56 + fir.rs:18-34, evaluated only at the kept instants)
//   rx_fast<DEC>: one workgroup = TS = 256*R output symbols.
//     1. streams the (TS+K-1)*DEC input samples it needs with 16-B loads, applies the
//        conjugate (or the reference's real) mix per sample and scatters them into DEC
//        polyphase planes in LDS  z_b[m] = z[m*DEC + D - b];
//     2. each lane computes R consecutive outputs  r_k = sum_b sum_t h[b+DEC*t] z_b[k-t]
//        with one sliding window per plane (ds_read_b64 per R complex MACs);
//     3. hard decision + store.
#include "modem_device.h"

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

// carrier.next() + pll.phase_offset (demodulator.rs:50): one f32 add, exact for offset 0
__device__ __forceinline__ float rx_phase(const RxParams& p, float carrier) {
#pragma clang fp contract(off)
    return carrier + p.phase_offset;
}

// x * e^{-j phase} (or the reference's x.re * (cos, -sin), demodulator.rs:46,53-54) for
// stream index n = nb + off (nb wave-uniform).
template <int MIX>
__device__ __forceinline__ float2 rx_mix(const RxParams& p, int64_t nb, int off, float2 x) {
    if (nb + off < 0) return make_float2(0.f, 0.f);   // before the stream: zero history
    float s, c;
    sincos_phase(rx_phase(p, carrier_phase_off(p.w, p.c0 + (uint64_t)nb, off, p.exact_idx)), s, c);
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
        const int si = (int)__builtin_fminf(__builtin_fmaxf(__builtin_rintf(fi), 0.f), (float)ms);
        const int sq = (int)__builtin_fminf(__builtin_fmaxf(__builtin_rintf(fq), 0.f), (float)ms);
        return (uint8_t)((si << p.bits_per_carrier) | sq);
    }
    return rx_slice_nearest(p, re, im);
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

// Rare path (first / last tile of a chunk, unaligned input, carrier index >= 2^53): one
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

// Steady state: every staged sample lies inside the chunk and below carrier index 2^53.
// Slot u of lane tid holds samples e = 2*(tid + NT*u) - PAR + {0,1}; the per-slot part of
// every index is a compile-time constant (NT*2/DEC plane elements per slot), so the LDS
// stores use immediate offsets and the phase needs one f64 add.
template <int DEC, typename InT, int MIX, int PAR, int U, int NT>
__device__ __forceinline__ void rx_stage_fast(const RxParams& p, float2* lds, int PS, int NS,
                                              double nbd, const typename InIO<InT>::Raw (&pre)[U]) {
    const int tid = threadIdx.x;
    // carrier index of the lane's first sample; opaque, so that the per-sample offsets stay
    // f64 literals instead of hoisted VGPR pairs
    double lb = nbd + (double)(2 * tid - PAR);
    asm volatile("" : "+v"(lb));
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
                s = 0.f; c = idx_f32(lb + (double)(j + 2 * NT * u));
#else
                sincos_phase(rx_phase(p, phase_from_f(p.w, idx_f32(lb + (double)(j + 2 * NT * u)))), s, c);
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
    const bool pf = p.x_aligned16 && p.exact_idx && NS + 1 <= 2 * NT * U;   // workgroup-uniform
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
            const double nbd = (double)(p.c0 + (uint64_t)(q_lo - (q_lo & 1) + p.n_start));
            if (q_lo & 1) rx_stage_fast<DEC, InT, MIX, 1, U, NT>(p, lds, PS, NS, nbd + 1.0, pre);
            else rx_stage_fast<DEC, InT, MIX, 0, U, NT>(p, lds, PS, NS, nbd, pre);
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
// Matched filter at the kept instants on the matrix cores (v_mfma_f32_16x16x32_f16):
//   rows i = 16 groups of 16 consecutive kept instants, cols c = instant in the group,
//   k = w = offset in a W = 32*NKS sample window ending at the group's last instant,
//   A[i][w] = z[start_i + w] (mixed input), B[w][c] = h[W - 1 - w - (15 - c)*DEC].
// Every real operand is split in two f16 halves, a = a_hi + a_lo (round to nearest), and
//   A*B ~= A_hi*B_hi + A_hi*B_lo + A_lo*B_hi      (dropped A_lo*B_lo < 2^-22 |a||b|)
// accumulates in f32: 6 MFMAs (re and im rails) per 32-sample k-step, 16x the MAC rate of
// the f32 MFMA. Range: the taps are scaled by 2^kb on the host (0 when their max is in [2^-3, 2^15)); the
// mixed samples of a tile are used as they are when the tile's max |z| lies in
// [2^-3, 2^15) (results then never depend on how a stream is cut into calls), and scaled
// by 2^ka into [2^14, 2^15) otherwise. Outputs are scaled back with ldexp (exact).
// LDS: four f16 planes (re_hi, re_lo, im_hi, im_lo) in natural sample order with 16 pad
// halves after every RW = 16*DEC samples (rxh_pos: conflict-free 16-B A reads), and NC shifted copies of the hi/lo reversed-tap table so that every lane's
// 8-tap B read is one aligned ds_read_b128.
template <int DEC, int NT_> struct RxMfmaCfg {
    static constexpr int NT = NT_;               // 64 (one wave) or 256 (4 waves)
    static constexpr int TS = NT / 64 * 256;     // kept instants per workgroup tile
    static constexpr int RW = 16 * DEC;          // samples per A row
    static constexpr int RP = RW + 16;           // padded row pitch (halves)
};
// Plane position of staged sample e: 16 pad halves after every RW samples. With the row pitch
// RW + 16 (= 2 mod 4 in 16-B units), the 16 lanes of each ds_read_b128 lane group (rows i at
// k-offset g, rows i' at g + 1) hit distinct bank quads; a pitch of RW + 8 was 2-way conflicted.
__host__ __device__ constexpr int rxh_pos(int e, int RW) { return e + 16 * (e / RW); }

// What the steady-state epilogue writes: baseband IQ, QAM-axis decisions, or both
// (RXE_GEN: any other combination, guarded per store).
enum { RXE_GEN = 0, RXE_IQ = 1, RXE_SYM = 2, RXE_IQSYM = 3, RXE_NEAREST = 4 };   // | NEAREST: LUT slicer

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

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));

// hi = rn_f16(v), lo = rn_f16(v - hi) for two values (v - hi is exact in f32).
__device__ __forceinline__ void split2(cf2 v, h2& hi, h2& lo) {
    hi = __builtin_convertvector(v, h2);
    float l0, l1;                                   // v - hi, exact: one v_fma_mix_f32 each
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(l0) : "v"(hi), "v"(v.x));
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(l1) : "v"(hi), "v"(v.y));
    lo = __builtin_convertvector((cf2){l0, l1}, h2);
}

// Conjugate mix of one sample, packed: (re, im) = (x*cs + y*sn, y*cs - x*sn) with the same
// roundings as fma(y, sn, x*cs) / fma(-x, sn, y*cs). cssn = (cs, sn). Written as vector ops
// (v_pk_mul_f32 + v_pk_fma_f32 with op_sel / neg modifiers), so that the compiler's hazard
// recognizer sees them and only pads where a transcendental's result is read too early.
__device__ __forceinline__ cf2 cmix(cf2 x, cf2 cssn) {
#ifdef MODEM_CMIX_ASM
    cf2 t, z;
    asm("s_nop 0\n\tv_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(t) : "v"(x), "v"(cssn));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[0,1,0]"
        : "=v"(z) : "v"(x), "v"(cssn), "v"(t));
    return z;
#else
    const cf2 t = x * cssn.xx;
    return __builtin_elementwise_fma(x.yx, (cf2){cssn.y, -cssn.y}, t);
#endif
}

// Four consecutive input samples (one lane's staging quad).
template <typename InT> struct Quad;
template <> struct Quad<float> {
    struct T { float4 a, b; };
    __device__ static T load(const void* x, int64_t q) {      // q: sample index (8-B aligned)
        const float4* v = reinterpret_cast<const float4*>(reinterpret_cast<const float2*>(x) + q);
#ifdef MODEM_RX_NT_LOAD
        const f32x4* w = reinterpret_cast<const f32x4*>(v);
        const f32x4 a = __builtin_nontemporal_load(w), b = __builtin_nontemporal_load(w + 1);
        return T{make_float4(a[0], a[1], a[2], a[3]), make_float4(b[0], b[1], b[2], b[3])};
#else
        return T{v[0], v[1]};
#endif
    }
    __device__ static void split(const T& t, float2 (&x)[4]) {
        x[0] = make_float2(t.a.x, t.a.y); x[1] = make_float2(t.a.z, t.a.w);
        x[2] = make_float2(t.b.x, t.b.y); x[3] = make_float2(t.b.z, t.b.w);
    }
};
template <> struct Quad<__half> {
    using T = uint4;
    __device__ static T load(const void* x, int64_t q) {
        return *reinterpret_cast<const uint4*>(reinterpret_cast<const __half2*>(x) + q);
    }
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

// Tile scale exponent from the lanes' max |z| (one barrier; red: 4 floats of LDS).
template <int NT>
__device__ __forceinline__ int tile_scale_exp(float lane_max, float* red) {
    float m = wave_max(lane_max);
    if (NT == 64) {
        __syncthreads();                                    // one wave: orders the LDS planes only
    } else {
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
        __syncthreads();
        m = __builtin_fmaxf(__builtin_fmaxf(red[0], red[1]), __builtin_fmaxf(red[2], red[3]));
    }
    const int ex = (int)((__float_as_uint(m) >> 23) & 0xff);
    if (ex >= 127 - 3 && ex < 127 + 15) return 0;          // max in [2^-3, 2^15): as is
    if (ex == 0 || ex == 0xff) return 0;                    // all zero / non-finite
    return 141 - ex;                                        // max * 2^k in [2^14, 2^15)
}

// The tiles one workgroup runs, in order: first, first + step, ... (count of them).
struct TileSeq { int64_t first, step, count; };

template <int DEC, int NKS, typename InT, int MIX, typename OutT, int NTT>
struct RxMfma {
    using C = RxMfmaCfg<DEC, NTT>;
    using Q = Quad<InT>;
    using QT = typename Q::T;
    static constexpr int NT = C::NT, TS = C::TS, RW = C::RW, RP = C::RP;
    static constexpr int W = 32 * NKS;
    static constexpr int NS = (TS - 16) * DEC + W;              // samples staged per tile
    static constexpr int NQ = (NS + 3) / 4;                     // quads
    static constexpr int U = (NQ + NT - 1) / NT;                // quads per lane
    // Plane layout. decim 4 (4 waves): unpadded, 16-B chunks XOR-swizzled within each aligned
    // group of 8 chunks — conflict-free A reads (tests/test_lds_banks.py) and 4 KiB less LDS
    // per workgroup than padding, which lets 4 workgroups share a CU. Otherwise rxh_pos.
#ifdef MODEM_RX_NOSWZ
    static constexpr bool SWZ = false;
#else
    static constexpr bool SWZ = DEC == 4 && NT == 256;
#endif
    __host__ __device__ static constexpr int ppos(int e) {    // plane position of staged sample e
        return SWZ ? ((((e >> 3) ^ (((e >> 7) & 3) << 1)) << 3) | (e & 7)) : rxh_pos(e, RW);
    }
    static constexpr int PL = SWZ ? (4 * NQ + 63) & ~63 : (rxh_pos(4 * NQ - 1, RW) + 1 + 7) & ~7;   // halves per plane
    static constexpr int NC = rx_mfma_table_copies(DEC);
    static constexpr int TB = rx_mfma_table_len(DEC, NKS);      // halves per table (hi or lo)
    static constexpr size_t LDS_BYTES = (size_t)4 * PL * 2 + (size_t)NC * 2 * TB * 2 + 16;   // + red
    static constexpr float GAIN = MIX == MIX_REFERENCE_REAL ? 2.0f : 1.0f;
    // Waves per SIMD the registers are held to: 4 for the swizzled layout (its LDS lets 4
    // workgroups share a CU; the matched filter then single-buffers its operands to fit 128
    // VGPRs: 35.0 vs 35.4 us on C3), else the compiler's choice (3 on C3).
#ifdef MODEM_RX_NOWPE
    static constexpr int WPE = 1;
#else
    static constexpr int WPE = SWZ && LDS_BYTES <= 40960 ? 4 : 1;
#endif
    static_assert((4 * NT) % RW == 0, "a staging slot spans whole rows");
    // plane offset between staging slots (the swizzle repeats every 1024 samples)
    static constexpr int SLOT_POS = SWZ ? 4 * NT : 4 * NT + 16 * (4 * NT / RW);

    // Rows hold 16 instants aligned to the absolute instant index (k % 16 == column), so an
    // instant's taps always fall at the same k positions of the 32-wide MFMA sums and the
    // result never depends on where a call starts. Tile t covers instants
    // kb + t*TS .., kb = k_first - lead; outputs before k_first are computed and dropped.
    __device__ static int lead(const RxParams& p) { return (int)(p.k_first & 15); }
    __device__ static int64_t q_lo_of(const RxParams& p, int64_t t) {
        return (p.k_first - lead(p) + t * TS) * DEC + p.D + 15 * DEC - W + 1 - p.n_start;
    }

    // Scale, split and write samples e0..e0+3 at plane offset o = rxh_pos(e0) (e0 % 4 == 0:
    // one row, 8-B aligned).
    __device__ static void put4o(_Float16* pl, int o, const float (&zr)[4], const float (&zi)[4], float sc) {
        h2 rh0, rl0, rh1, rl1, ih0, il0, ih1, il1;
        split2((cf2){zr[0], zr[1]} * sc, rh0, rl0);
        split2((cf2){zr[2], zr[3]} * sc, rh1, rl1);
        split2((cf2){zi[0], zi[1]} * sc, ih0, il0);
        split2((cf2){zi[2], zi[3]} * sc, ih1, il1);
        *reinterpret_cast<h4*>(pl + o) = (h4){rh0.x, rh0.y, rh1.x, rh1.y};
        *reinterpret_cast<h4*>(pl + PL + o) = (h4){rl0.x, rl0.y, rl1.x, rl1.y};
        *reinterpret_cast<h4*>(pl + 2 * PL + o) = (h4){ih0.x, ih0.y, ih1.x, ih1.y};
        *reinterpret_cast<h4*>(pl + 3 * PL + o) = (h4){il0.x, il0.y, il1.x, il1.y};
    }

    // Steady state: the tile's samples lie inside the chunk, carrier index < 2^53. Staged
    // at scale 1 (the tile max is tracked on the way). Returns the tile's scale exponent: 0,
    // or for a tile whose max falls outside [2^-3, 2^15) the exponent the general path
    // (stage_slow) must restage it with.
    // Load staging slot u of the tile whose window starts at chunk sample `base` (clamped
    // into the chunk by the caller); l0 = 4 * lane, opaque.
    __device__ static QT load_slot(const RxParams& p, int64_t base, int l0, int u) {
        int e0 = l0 + 4 * NT * u;
        if ((u + 1) * NT > NQ) e0 = e0 < 4 * (NQ - 1) ? e0 : 4 * (NQ - 1);   // spare lanes
#ifdef MODEM_ABLATE_LOAD
        float v = 0.5f + 1e-3f * (float)(e0 & 7);   // in the f16 window: no restaging
        asm volatile("" : "+v"(v));
        if constexpr (std::is_same<InT, float>::value) return QT{make_float4(v, v, v, v), make_float4(v, v, v, v)};
        else return make_uint4(__float_as_uint(v), 0, 0, 0);
#else
        return Q::load(p.x, base + e0);
#endif
    }

    // Steady-state staging of one tile from the prefetched registers `pre`. (Reloading each
    // slot for the next tile right after it is consumed, to give the loads a whole tile period,
    // measured 1 us slower on C3 than prefetching after the stage.)
    __device__ static int stage_fast(const RxParams& p, _Float16* pl, float* red, double nbd,
                                     const QT (&pre)[U]) {
        const int tid = threadIdx.x;
        // carrier index of the lane's first sample; opaque, so that the per-sample offsets
        // stay immediates instead of 4*U hoisted loop-invariant VGPRs
        double lb = nbd + (double)(4 * tid);
        int pos0 = ppos(4 * tid);                         // slot u writes at pos0 + u * SLOT_POS
        asm volatile("" : "+v"(lb), "+v"(pos0));
        const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        float mx = 0.f;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            // the last slot is partial: only the waves that own some of its quads run it
            if ((u + 1) * NT > NQ && 64 * wave + NT * u >= NQ) continue;   // wave-uniform
            float2 x[4];
            Q::split(pre[u], x);
            const int e0 = 4 * (tid + NT * u);
            float zr[4], zi[4];
            // the quad's phases as two packed pairs, computed side by side (independent
            // chains fill each other's VALU dependency wait states)
            cf2 sn2[2], cs2[2];
            {
                const cf2 nf0 = (cf2){idx_f32(lb + (double)(4 * NT * u)), idx_f32(lb + (double)(4 * NT * u + 1))};
                const cf2 nf1 = (cf2){idx_f32(lb + (double)(4 * NT * u + 2)), idx_f32(lb + (double)(4 * NT * u + 3))};
#ifdef MODEM_ABLATE_MIX
                sn2[0] = sn2[1] = (cf2){0.f, 0.f}; cs2[0] = nf0; cs2[1] = nf1;
#else
                // rx_phase: one add on the packed phases (no product to contract)
                const cf2 ph0 = phase_from_f2(p.w, nf0) + p.phase_offset;
                const cf2 ph1 = phase_from_f2(p.w, nf1) + p.phase_offset;
                sincos_phase2(ph0, sn2[0], cs2[0]);
                sincos_phase2(ph1, sn2[1], cs2[1]);
#endif
            }
#pragma unroll
            for (int j = 0; j < 4; j += 2) {
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const float sn = sn2[j / 2][i], cs = cs2[j / 2][i];
                    if (MIX == MIX_REFERENCE_REAL) { zr[j + i] = x[j + i].x * cs; zi[j + i] = x[j + i].x * -sn; }
                    else {
                        const cf2 z = cmix((cf2){x[j + i].x, x[j + i].y}, (cf2){cs, sn});
                        zr[j + i] = z.x; zi[j + i] = z.y;
                    }
                    // only the last slot can reach past the tile: its extra samples are not counted
                    if ((u + 1) * 4 * NT <= NS || e0 + j + i < NS)      // one v_max3 per sample
                        asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(mx) : "v"(zr[j + i]), "v"(zi[j + i]));
                }
            }
#ifdef MODEM_ABLATE_PUT
            asm volatile("" :: "v"(zr[0]), "v"(zr[1]), "v"(zr[2]), "v"(zr[3]), "v"(zi[0]), "v"(zi[1]), "v"(zi[2]), "v"(zi[3]));
#else
            if ((u + 1) * 4 * NT <= NS || e0 < NS) put4o(pl, pos0 + u * SLOT_POS, zr, zi, 1.0f);
#endif
            __builtin_amdgcn_sched_barrier(0);              // one quad's temporaries at a time
        }
        // ka != 0 (rare: out-of-window magnitudes): the caller restages the tile scaled
#ifdef MODEM_ABLATE_TMAX
        asm volatile("" :: "v"(mx));
        __syncthreads();
        return 0;
#endif
        return tile_scale_exp<NT>(mx, red);
    }

    // First / last tiles of a chunk, unaligned input, carrier index >= 2^53: per sample, two
    // passes (max, then scale + split).
    __device__ static int stage_slow(const RxParams& p, _Float16* pl, float* red, int64_t q_lo) {
        const int64_t n_lo = q_lo + p.n_start;
        float mx = 0.f;
        for (int e0 = 4 * threadIdx.x; e0 < NS; e0 += 4 * NT)
            for (int j = 0; j < 4 && e0 + j < NS; ++j) {
                const float2 z = rx_mix<MIX>(p, n_lo, e0 + j, rx_sample<InT>(p, q_lo + e0 + j));
                mx = __builtin_fmaxf(mx, __builtin_fmaxf(__builtin_fabsf(z.x), __builtin_fabsf(z.y)));
            }
        const int ka = tile_scale_exp<NT>(mx, red);
        const float sc = __builtin_ldexpf(1.0f, ka < -126 ? -126 : (ka > 127 ? 127 : ka));
        for (int e0 = 4 * threadIdx.x; e0 < NS; e0 += 4 * NT) {
            float zr[4], zi[4];
            for (int j = 0; j < 4; ++j) {
                const float2 z = e0 + j < NS ? rx_mix<MIX>(p, n_lo, e0 + j, rx_sample<InT>(p, q_lo + e0 + j))
                                             : make_float2(0.f, 0.f);
                zr[j] = z.x; zi[j] = z.y;
            }
            put4o(pl, ppos(e0), zr, zi, sc);
        }
        return ka;
    }

    // One 16x16 tile per wave. Lane (i = lane & 15, g = lane >> 4) reads A row i, samples
    // 32s + 8g .. +7, and B[32s + 8g + j][c = i] = T[32s + 8g + j + (15 - c)*DEC].
    __device__ static void fir(const _Float16* pl, const _Float16* tbl, f32x4& dre, f32x4& dim) {
        const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        const int i = lane & 15, g = lane >> 4;
        const _Float16* arow = pl + (16 * wave + i) * RP + 8 * g;
        const int ae = (16 * wave + i) * RW + 8 * g;            // sample of this lane's first A read
        const int xb = 8 * g + (15 - i) * DEC;                  // B start for this lane's column
        const int q = xb & 7;                                   // copy with Tq[y] = T[y + q]
        const _Float16* brow = tbl + (q / (8 / NC)) * 2 * TB + (xb - q);
#ifdef MODEM_ABLATE_FIR
        const h8 a0 = *reinterpret_cast<const h8*>(arow);
        dre = (f32x4){(float)a0[0], 0.f, 0.f, 0.f};
        dim = (f32x4){(float)brow[0], 0.f, 0.f, 0.f};
        return;
#endif
        f32x4 r0 = {0.f, 0.f, 0.f, 0.f}, m0 = r0;     // one accumulator per rail
        auto aoff = [](int s) { return 32 * s + 16 * ((32 * s) / RW); };
        h8 a[2][4], b[2][2];
        auto load = [&](int s, int slot) {
            const _Float16* ap = SWZ ? pl + ppos(ae + 32 * s) : arow + aoff(s);
            a[slot][0] = *reinterpret_cast<const h8*>(ap);
            a[slot][1] = *reinterpret_cast<const h8*>(ap + PL);
            a[slot][2] = *reinterpret_cast<const h8*>(ap + 2 * PL);
            a[slot][3] = *reinterpret_cast<const h8*>(ap + 3 * PL);
            b[slot][0] = *reinterpret_cast<const h8*>(brow + 32 * s);
            b[slot][1] = *reinterpret_cast<const h8*>(brow + TB + 32 * s);
        };
        // WPE 4: single-buffered operands (fewer registers; the other waves hide the LDS
        // latency); otherwise the next k-step's operands load during this one's products
        if (WPE < 4) load(0, 0);
#pragma unroll
        for (int s = 0; s < NKS; ++s) {
            const int c = WPE < 4 ? s & 1 : 0;
            if (WPE >= 4) load(s, 0);
            else if (s + 1 < NKS) load(s + 1, c ^ 1);
            r0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[c][0], b[c][0], r0, 0, 0, 0);
            m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[c][2], b[c][0], m0, 0, 0, 0);
            r0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[c][0], b[c][1], r0, 0, 0, 0);
            m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[c][2], b[c][1], m0, 0, 0, 0);
            r0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[c][1], b[c][0], r0, 0, 0, 0);
            m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[c][3], b[c][0], m0, 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
        dre = r0;
        dim = m0;
    }

    // D[row][col]: row = 4*(lane>>4) + r, col = lane&15 -> instant ot + 16*row + col.
    template <int EM>
    __device__ static void emit_full(const RxParams& p, int64_t ot, const f32x4& dre, const f32x4& dim, int kab) {
        const int lane = threadIdx.x & 63;
#ifdef MODEM_ABLATE_STORE
#pragma unroll
        for (int r = 0; r < 4; ++r) asm volatile("" :: "v"(dre[r]), "v"(dim[r]));
        return;
#endif
        // uniform base pointers + 32-bit lane offsets: saddr + voffset stores, no 64-bit
        // per-lane address registers
        OutT* qb = reinterpret_cast<OutT*>(p.out_iq) + 2 * ot;
        uint8_t* sb = p.out_sym + ot;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t off = (uint32_t)(16 * (4 * (lane >> 4) + r) + (lane & 15));
            float re = dre[r], im = dim[r];
            if (kab != 0) { re = __builtin_ldexpf(re, -kab); im = __builtin_ldexpf(im, -kab); }   // uniform
            re *= GAIN;
            im *= GAIN;
            if (EM == RXE_GEN) {
                rx_emit<OutT>(p, ot + off, re, im);
                continue;
            }
            if (EM & RXE_IQ) OutIO<OutT>::store_one(qb, off, re, im);
            if (EM & RXE_SYM)
                sb[off] = !(EM & RXE_NEAREST) ? rx_slice_qam(p, re, im)
                        : p.bps == 2 ? rx_slice_nearest4(p, re, im) : rx_slice_nearest(p, re, im);
        }
    }

    __device__ static void emit_edge(const RxParams& p, int64_t ot, const f32x4& dre, const f32x4& dim, int kab) {
        const int lane = threadIdx.x & 63;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t o = ot + 16 * (4 * (lane >> 4) + r) + (lane & 15);
            if (o >= 0 && o < p.nout)
                rx_emit<OutT>(p, o, GAIN * __builtin_ldexpf(dre[r], -kab), GAIN * __builtin_ldexpf(dim[r], -kab));
        }
    }

    // The tiles of `sq` (the XCD-matched top-down rounds of rx_mfma_body; a contiguous range
    // per workgroup measured 9 % faster on C3 than bottom-up rounds, and dynamic tile handout
    // through per-XCD atomic counters did not beat it either). When the input is 8-B aligned
    // and the carrier indices stay below 2^53, the run of "full" tiles (all staged samples
    // inside the chunk, all 1024 instants kept) goes through the prefetched loop, whose
    // epilogue EM stores unconditionally; the first and last tiles of the chunk take the
    // general path.
    template <int EM>
    __device__ static void run(const RxParams& p, _Float16* pl, const _Float16* tbl, float* red,
                               const TileSeq sq) {
        const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // scalar
        // quad loads need dword alignment only (16-B loads at 8-B aligned sample offsets)
        const bool fast = p.exact_idx && ((uintptr_t)p.x & 3) == 0;
        const int kb = p.tap_scale_exp;
        const int ld = lead(p);
        auto full = [&](int64_t t) {
            const int64_t q = q_lo_of(p, t);
            return fast && q >= 0 && q + 4 * NQ <= p.N && t * TS >= ld && (t + 1) * TS - ld <= p.nout;
        };
        QT pre[U];
        // Base clamped into the chunk; issued when this workgroup has a next tile (a non-full
        // next tile is restaged). The epilogue's stores stay unconditional, so the next trip's
        // vmcnt waits remain counted.
        auto clamped_base = [&](int64_t t) {
            const int64_t base = q_lo_of(p, t);   // (the first tile of a call may start before 0)
            return base > p.N - 4 * NQ ? p.N - 4 * NQ : base < 0 ? 0 : base;
        };
        auto prefetch = [&](int64_t t) {
            const int64_t base = clamped_base(t);
            int l0 = 4 * tid;                               // opaque: no per-slot hoisted addresses
            asm volatile("" : "+v"(l0));
#pragma unroll
            for (int u = 0; u < U; ++u)                     // the partial last slot: its waves only
                if ((u + 1) * NT <= NQ || 64 * wave + NT * u < NQ) pre[u] = load_slot(p, base, l0, u);
        };
        int64_t i = 0, t = sq.first;
        bool restage = false;
        STAMP_DECL;
        while (i < sq.count) {
            if (full(t) && !restage) {
                prefetch(t);
                for (; i < sq.count && full(t); ++i, t += sq.step) {
                    const int64_t n_lo = q_lo_of(p, t) + p.n_start;
#ifdef MODEM_STAMPS
                    STAMP(0);                              // loop overhead
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    STAMP(1);                              // waiting for the tile's samples
#endif
                    const int ka = stage_fast(p, pl, red, (double)(p.c0 + (uint64_t)n_lo), pre);
                    STAMP(2);                              // staging + tile-max barrier
                    if (ka != 0) { restage = true; break; }       // uniform; leaves the loop
                    // (the tile-max reduction in stage_fast ended with a barrier: planes visible)
                    if (i + 1 < sq.count) prefetch(t + sq.step);   // next samples fly during the MFMAs
                    STAMP(3);                              // prefetch issue
                    f32x4 dre, dim;
                    fir(pl, tbl, dre, dim);
                    STAMP(4);                              // matched filter
                    emit_full<EM>(p, t * TS + wave * 256 - ld, dre, dim, kb);
                    STAMP(5);                              // epilogue
                    __syncthreads();                       // LDS is restaged next trip
                    STAMP(6);                              // end barrier
                }
            } else {
                __syncthreads();                           // `red` and the planes are reused
                restage = false;
                const int ka = stage_slow(p, pl, red, q_lo_of(p, t));
                __syncthreads();
                f32x4 dre, dim;
                fir(pl, tbl, dre, dim);
                emit_edge(p, t * TS + wave * 256 - ld, dre, dim, ka + kb);
                __syncthreads();
                ++i;
                t += sq.step;
                STAMP(7);                                  // general-path tiles
            }
        }
        STAMP_FLUSH(blockIdx.x * (NT / 64) + wave);
    }

};

// (Capping this kernel at 4 waves/SIMD fits the steady loop in 128 registers but measured
// slower on C3: 41.6 vs 35.7 us, with LDS still holding it at 3 workgroups per CU.)
// One channel's share of a launch: workgroup `bid` of `nb` working on channel p.
template <int DEC, int NKS, typename InT, int MIX, typename OutT, int NT>
__device__ __forceinline__ void rx_mfma_body(const RxParams& p, const _Float16* __restrict__ tables,
                                             int64_t bid, int64_t nb) {
    using K = RxMfma<DEC, NKS, InT, MIX, OutT, NT>;
    extern __shared__ __attribute__((aligned(16))) _Float16 lds_h[];
    _Float16* pl = lds_h;                                   // 4 sample planes
    _Float16* tbl = lds_h + 4 * K::PL;                      // NC x (hi, lo) tap tables
    float* red = reinterpret_cast<float*>(tbl + K::NC * 2 * K::TB);
    if (bid == 0) rx_state_update<InT>(p);
    for (int j = threadIdx.x; j < K::NC * 2 * K::TB / 8; j += K::NT)
        reinterpret_cast<h8*>(tbl)[j] = reinterpret_cast<const h8*>(tables)[j];
    __syncthreads();
    const int64_t ntiles = (p.nout + K::lead(p) + K::TS - 1) / K::TS;
#ifndef MODEM_RX_CONTIG
    // Rounds of nb tiles from the top down, tile R - (r + 1) nb + bid in round r. The TX hands
    // its tiles out grid-strided (tile i to workgroup i mod grid, both grids multiples of 8, so
    // tile i is written on XCD slot i mod 8); the RX's first round then reads the ~32 MiB the
    // TX wrote last, each tile on the XCD slot that wrote it (blocks b and b + 8 share an XCD).
    // C3: 35.0 -> 33.8 us, A/B twice on one box against contiguous ranges per workgroup
    // (MODEM_RX_CONTIG; that variant now spills 28 B/lane, 37-38 us). The XCD match is what
    // pays: the same rounds with the slots shifted by 1 or 4 (MODEM_RX_XCD_SHIFT) measured
    // 38.1-39.1 us. PMC FETCH_SIZE per launch is unchanged (139 vs 137 MB).
    const int64_t R = (ntiles + nb - 1) / nb * nb;
#ifdef MODEM_RX_XCD_SHIFT     // experiment: the same rounds with the XCD slots mismatched
    TileSeq sq{R - nb + (bid + MODEM_RX_XCD_SHIFT) % nb, -nb, R / nb};
#else
    TileSeq sq{R - nb + bid, -nb, R / nb};
#endif
    if (sq.first >= ntiles) { sq.first -= nb; --sq.count; }
#else
    const int64_t t0 = ntiles * bid / nb, t1 = ntiles * (bid + 1) / nb;
    const TileSeq sq{t0, 1, t1 - t0};
#endif
    if (sq.count <= 0) return;
#ifdef MODEM_STAGGER
    // workgroups dealt to the same CU (b, b + CUs, ...) start a fraction of a tile apart so
    // their staging (VALU) and matrix phases interleave instead of running in lockstep
    {
        const int k = (int)(bid / MODEM_STAGGER) % 3;
        for (int i = 0; i < k * 12; ++i) __builtin_amdgcn_s_sleep(127);   // ~8K cycles each step
    }
#endif
    // f32 input with the complex mix (the loopback chain): the epilogue is specialised on what
    // it stores, so the tile loop's store count is static. Other variants share the guarded one.
    if (std::is_same<InT, float>::value && MIX == MIX_COMPLEX) {
        const bool qam = p.slicer_kind == SLICER_QAM_AXIS && p.out_sym;
        if (p.out_iq && qam) { K::template run<RXE_IQSYM>(p, pl, tbl, red, sq); return; }
        if (p.out_iq && p.out_sym && p.slicer_kind == SLICER_NEAREST) {
            K::template run<RXE_IQSYM | RXE_NEAREST>(p, pl, tbl, red, sq);
            return;
        }
        if (p.out_iq && !p.out_sym) { K::template run<RXE_IQ>(p, pl, tbl, red, sq); return; }
        if (!p.out_iq && qam) { K::template run<RXE_SYM>(p, pl, tbl, red, sq); return; }
    }
    // f16 storage of the loopback chain (C5 f16): I/Q and QAM decisions, unconditional stores
    if (std::is_same<InT, __half>::value && MIX == MIX_COMPLEX && p.out_iq && p.out_sym &&
        p.slicer_kind == SLICER_QAM_AXIS) {
        K::template run<RXE_IQSYM>(p, pl, tbl, red, sq);
        return;
    }
    K::template run<RXE_GEN>(p, pl, tbl, red, sq);
}

template <int DEC, int NKS, typename InT, int MIX, typename OutT, int NT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(RxMfma<DEC, NKS, InT, MIX, OutT, NT>::WPE)))
void rx_mfma(const RxParams p, const _Float16* __restrict__ tables) {
    rx_mfma_body<DEC, NKS, InT, MIX, OutT, NT>(p, tables, blockIdx.x, gridDim.x);
}

// A batch of independent channels of one configuration (modem_rx_process_batch): workgroup
// b serves channel b / g as its workgroup b % g of g.
template <int DEC, int NKS, typename InT, int MIX, typename OutT, int NT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(RxMfma<DEC, NKS, InT, MIX, OutT, NT>::WPE)))
void rx_mfma_batch(const RxBatch b, const _Float16* __restrict__ tables) {
#ifdef MODEM_BATCH_INTERLEAVE
    const int ch = (int)(blockIdx.x % (unsigned)b.nch);
    const unsigned bid = blockIdx.x / (unsigned)b.nch;
#else
    const int ch = (int)(blockIdx.x / (unsigned)b.g);
    const unsigned bid = blockIdx.x - (unsigned)ch * b.g;
#endif
    const RxParams p = b.p[ch];     // one bulk copy: the body's uses read registers, not kernarg
    rx_mfma_body<DEC, NKS, InT, MIX, OutT, NT>(p, tables, bid, b.g);
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

template <int DEC, int NKS, typename InT, int MIX, typename OutT, int NT>
static hipError_t rxm_go_nt(const RxParams& p, const void* tables, hipStream_t s) {
    using K = RxMfma<DEC, NKS, InT, MIX, OutT, NT>;
    const int64_t ntiles = (p.nout + (p.k_first & 15) + K::TS - 1) / K::TS;
    const size_t lds = K::LDS_BYTES;
    const void* k = reinterpret_cast<const void*>(&rx_mfma<DEC, NKS, InT, MIX, OutT, NT>);
    static const int cap = env_wgs_per_cu("MODEM_RX_WGS_PER_CU");
    hipLaunchKernelGGL((rx_mfma<DEC, NKS, InT, MIX, OutT, NT>), dim3(persistent_grid(k, K::NT, lds, ntiles, cap)),
                       dim3(K::NT), lds, s, p, static_cast<const _Float16*>(tables));
    return hipGetLastError();
}

template <int DEC, int NKS, typename InT, int MIX, typename OutT>
static hipError_t rxm_go(const RxParams& p, const void* tables, hipStream_t s) {
#ifdef MODEM_RX_NT64
    return rxm_go_nt<DEC, NKS, InT, MIX, OutT, 64>(p, tables, s);
#else
    return rxm_go_nt<DEC, NKS, InT, MIX, OutT, 256>(p, tables, s);
#endif
}

template <int DEC, int NKS, typename InT, typename OutT>
static hipError_t rxm_go_batch(RxBatch b, const void* tables, hipStream_t s) {
    using K = RxMfma<DEC, NKS, InT, MIX_COMPLEX, OutT, 256>;
    int64_t ntiles = 0;
    for (int c = 0; c < b.nch; ++c) {
        const int64_t t = (b.p[c].nout + (b.p[c].k_first & 15) + K::TS - 1) / K::TS;
        ntiles = t > ntiles ? t : ntiles;
    }
    const size_t lds = K::LDS_BYTES;
    const void* k = reinterpret_cast<const void*>(&rx_mfma_batch<DEC, NKS, InT, MIX_COMPLEX, OutT, 256>);
    const int64_t cap = persistent_grid(k, K::NT, lds, INT64_MAX);
    int64_t g = cap / b.nch;
    g = g < 1 ? 1 : g > ntiles ? (ntiles > 0 ? ntiles : 1) : g;
    b.g = (int32_t)g;
    hipLaunchKernelGGL((rx_mfma_batch<DEC, NKS, InT, MIX_COMPLEX, OutT, 256>), dim3((unsigned)(g * b.nch)),
                       dim3(K::NT), lds, s, b, static_cast<const _Float16*>(tables));
    return hipGetLastError();
}

// (decim, k-steps) variants: W = 32 * nks >= 15 * decim + ntaps.
#ifdef MODEM_DEV_MIN      // experiment builds: the C3 variant only
#define RXM_TABLE(X) X(4, 6)
#else
#define RXM_TABLE(X) X(2, 2) X(2, 3) X(2, 5) X(2, 8) X(4, 3) X(4, 4) X(4, 6) X(4, 8) X(8, 5) X(8, 6) X(8, 9) X(8, 20)
#endif

template <typename InT, int MIX, typename OutT>
static hipError_t rxm_sel(const RxParams& p, int decim, int nks, const void* tables, hipStream_t s) {
#define RXM(D, N) if (decim == D && nks == N) return rxm_go<D, N, InT, MIX, OutT>(p, tables, s);
    RXM_TABLE(RXM)
#undef RXM
    return hipErrorInvalidValue;
}

template <typename T>
static hipError_t rxm_sel_batch(const RxBatch& b, int decim, int nks, const void* tables, hipStream_t s) {
#define RXM(D, N) if (decim == D && nks == N) return rxm_go_batch<D, N, T, T>(b, tables, s);
    RXM_TABLE(RXM)
#undef RXM
    return hipErrorInvalidValue;
}

hipError_t launch_rx_mfma_batch(const RxBatch& b, int decim, int nks, const void* tables, int dtype,
                                hipStream_t s) {
    if (b.nch < 1 || b.nch > kBatchMax) return hipErrorInvalidValue;
#ifdef MODEM_DEV_MIN
    if (dtype != 0) return hipErrorInvalidValue;
    return rxm_sel_batch<float>(b, decim, nks, tables, s);
#endif
    return dtype == 1 ? rxm_sel_batch<__half>(b, decim, nks, tables, s) : rxm_sel_batch<float>(b, decim, nks, tables, s);
}

int rx_mfma_ksteps(int decim, int L) {
    const int need = (15 * decim + L + 31) / 32;
    int best = 0;
#define RXK(D, N) if (decim == D && N >= need && (best == 0 || N < best)) best = N;
    RXM_TABLE(RXK)
#undef RXK
    return best;
}

hipError_t launch_rx_mfma(const RxParams& p, int decim, int nks, const void* tables, int in_dtype,
                          int out_dtype, int mix, hipStream_t s) {
#ifdef MODEM_DEV_MIN
    if (in_dtype != 0 || out_dtype != 0 || mix != MIX_COMPLEX) return hipErrorInvalidValue;
    return rxm_sel<float, MIX_COMPLEX, float>(p, decim, nks, tables, s);
#endif
    auto go = [&](auto in_t, auto out_t) {
        using InT = decltype(in_t);
        using OutT = decltype(out_t);
        return mix == MIX_REFERENCE_REAL ? rxm_sel<InT, MIX_REFERENCE_REAL, OutT>(p, decim, nks, tables, s)
                                         : rxm_sel<InT, MIX_COMPLEX, OutT>(p, decim, nks, tables, s);
    };
    if (in_dtype == 1) return out_dtype == 1 ? go(__half(), __half()) : go(__half(), float());
    return out_dtype == 1 ? go(float(), __half()) : go(float(), float());
}

hipError_t launch_rx(const RxParams& p, int decim, int in_dtype, int out_dtype, int mix,
                     hipStream_t s) {
#ifdef MODEM_DEV_MIN
    return hipErrorInvalidValue;
#endif
    if (in_dtype == 1)
        return out_dtype == 1 ? rx_mixsel<__half, __half>(p, decim, mix, s)
                              : rx_mixsel<__half, float>(p, decim, mix, s);
    return out_dtype == 1 ? rx_mixsel<float, __half>(p, decim, mix, s)
                          : rx_mixsel<float, float>(p, decim, mix, s);
}


}  // namespace mk

#ifdef MODEM_STAMPS
// Diagnostic builds only (tools/stamps.py): the per-wave segment cycle sums of the stamped
// RX launches (same translation unit as the kernel that writes them).
extern "C" int modem_debug_stamps(unsigned long long* host, size_t n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(mk::g_stamps), n * sizeof(unsigned long long)) == hipSuccess ? 0 : -3;
}
#endif
