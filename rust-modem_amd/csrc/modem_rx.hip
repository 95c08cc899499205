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
#include "modem_rx_mfma.h"
#include "modem_variants.h"

namespace mk {

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
                rx_sincos(p, phase_from_f(p.w, idx_f32(lb + (double)(j + 2 * NT * u))), s, c);
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

// Bit-exact reference demodulator (MODEM_MIX_REFERENCE_REAL_EXACT; demodulator.rs:44-56 at the
// kept instants): every f32 operation of the reference in its order. Per staged sample
// phase = Carrier::next() + pll.phase_offset (one f32 add), (c, s) = glibc's cosf / sinf
// (lm::, the library Rust's f32::cos / sin call), z = (x.re * c, x.re * -s); per output the
// FIRFilter::calc fold (fir.rs:18-34) s = ((0 + z[n] h0) + z[n-1] h1) + ..., separate multiply
// and add, over a history that is zero before the stream; y = 2 s. Thread per kept instant,
// ts instants per workgroup, their (ts - 1) * decim + L mixed samples in LDS.
template <typename InT, typename OutT>
__global__ __launch_bounds__(256) void rx_exact(const RxParams p, int ts) {
#pragma clang fp contract(off)
    extern __shared__ __attribute__((aligned(16))) float2 zl[];
    const int L = p.L, DEC = p.decim;
    if (blockIdx.x == 0) rx_state_update<InT>(p);
    const int64_t o0 = (int64_t)blockIdx.x * ts;
    if (o0 >= p.nout) return;
    const int64_t n_lo = (p.k_first + o0) * DEC + p.D - (L - 1);      // stream index of zl[0]
    const int NS = (ts - 1) * DEC + L;
    for (int e = threadIdx.x; e < NS; e += blockDim.x) {
        const int64_t n = n_lo + e;
        float2 z = make_float2(0.f, 0.f);                              // history before the stream
        if (n >= 0) {
            const float x = rx_sample<InT>(p, n - p.n_start).x;       // Complex::re
            const float ph = rx_phase(p, carrier_phase(p.w, p.c0 + (uint64_t)n, p.exact_idx));
            z = make_float2(x * lm::cosf<true>(ph), x * -lm::sinf<true>(ph));
        }
        zl[e] = z;
    }
    __syncthreads();
    const int j = threadIdx.x;
    if (j >= ts || o0 + j >= p.nout) return;
    const float2* zc = zl + j * DEC + (L - 1);                         // the instant's newest sample
    float si = 0.f, sq = 0.f;
    for (int t = 0; t < L; ++t) {
        const float h = p.taps[(t % DEC) * p.K + t / DEC];            // h[t] (polyphase layout)
        si = si + zc[-t].x * h;
        sq = sq + zc[-t].y * h;
    }
    rx_emit<OutT>(p, o0 + j, 2.0f * si, 2.0f * sq);
}

template <typename InT, typename OutT>
static hipError_t rx_exact_go(const RxParams& p, hipStream_t s) {
    int ts = 256;
    while (ts > 1 && (size_t)((ts - 1) * p.decim + p.L) * sizeof(float2) > 65536) ts /= 2;
    const size_t lds = (size_t)((ts - 1) * p.decim + p.L) * sizeof(float2);
    if (lds > 65536) return hipErrorInvalidValue;
    const int64_t nblk = (p.nout + ts - 1) / ts;
    hipLaunchKernelGGL((rx_exact<InT, OutT>), dim3((unsigned)(nblk > 0 ? nblk : 1)), dim3(256), lds, s, p, ts);
    return hipGetLastError();
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


// The matrix-core variants are instantiated in their own translation units (modem_rxm_*.hip,
// by element types: the sources compile in parallel); here only their dispatch.
hipError_t launch_rx_mfma_batch(const RxBatch& b, int decim, int nks, const void* tables, int dtype,
                                hipStream_t s) {
    if (b.nch < 1 || b.nch > kBatchMax) return hipErrorInvalidValue;
    return dtype == 1 ? rxm_sel_batch<__half>(b, decim, nks, tables, s) : rxm_sel_batch<float>(b, decim, nks, tables, s);
}

int rx_mfma_ksteps(int decim, int L) {
    const int need = (15 * decim + L + 31) / 32;
    int best = 0;
#define RXK(D, N) if (decim == D && N >= need && (best == 0 || N < best)) best = N;
    MODEM_RXM_TABLE(RXK)
#undef RXK
    return best;
}

hipError_t launch_rx_mfma(const RxParams& p, int decim, int nks, const void* tables, int in_dtype,
                          int out_dtype, int mix, hipStream_t s) {
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
    if (mix == MIX_REFERENCE_REAL_EXACT) {
        auto go = [&](auto in_t) {
            using InT = decltype(in_t);
            return out_dtype == 1 ? rx_exact_go<InT, __half>(p, s) : rx_exact_go<InT, float>(p, s);
        };
        return in_dtype == 2 ? go(int16_t()) : in_dtype == 1 ? go(__half()) : go(float());
    }
    if (in_dtype == 2) return hipErrorInvalidValue;
    if (in_dtype == 1)
        return out_dtype == 1 ? rx_mixsel<__half, __half>(p, decim, mix, s)
                              : rx_mixsel<__half, float>(p, decim, mix, s);
    return out_dtype == 1 ? rx_mixsel<float, __half>(p, decim, mix, s)
                          : rx_mixsel<float, float>(p, decim, mix, s);
}

}  // namespace mk
