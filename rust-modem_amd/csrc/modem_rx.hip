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
        // Base clamped into the chunk; issued when this workgroup has a next tile (a non-full
        // next tile is restaged). The epilogue's stores stay unconditional, so the next trip's
        // vmcnt waits remain counted.
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
                    if (t + 1 < t1) prefetch(t + 1);       // next samples fly during the MFMAs
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


}  // namespace mk
