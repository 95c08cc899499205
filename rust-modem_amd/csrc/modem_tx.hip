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
#include "modem_tx_mfma.h"
#include "modem_variants.h"

namespace mk {

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
    if (OUT_MODE != OUT_IQ_BASEBAND) {
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

// mod_trig (util.rs:3-6: x - TWO_PI * floor(x / TWO_PI), the quotient an IEEE f32 division) for
// any f32 (the scan's phases can be negative), without the division: the carrier's division-free
// floor (phase_from_f: q0 = x RC, r = fma(-q0, TWO_PI, x), q1 = fma(r, RC, q0)) gives the same
// result bit for bit for every finite f32 once -0 is mapped to +0 (x + 0: the identity elsewhere;
// the reference gives +0 for -0, the division-free form -0). tools/mod_trig_check.cpp checks all
// 2^32 inputs: 0 mismatches. The IEEE division was ~11 dependent instructions of the scans' serial
// step (profiles/r06_scan_rate.txt).
__device__ __forceinline__ float mod_trig_ieee(float x) {
#pragma clang fp contract(off)
    const float xz = x + 0.0f;
    const float q0 = xz * kRcp2Pi;
    const float r = __builtin_fmaf(-q0, kTwoPi, xz);
    const float q1 = __builtin_fmaf(r, kRcp2Pi, q0);
    return xz - kTwoPi * __builtin_floorf(q1);
}

// DMPSK / MFSK / BFSK: update() runs at every symbol tick (modulator.rs:90-93) with the
// phase carried in f32 from symbol to symbol, so the states are a serial recurrence (no exact
// parallel form: the reachable f32 states do not close). One step, the reference's
// f32 operations in its order:
//   DMPSK (dmpsk.rs:29-33): phase = mod_trig(phase + sym * shift)
//   MFSK (mfsk.rs:68-75):   off = mod_trig(off + (cur - next) * dev * s); cur = next
//   BFSK (bfsk.rs:42-53):   on a change of bit, phase = mod_trig(phase + (b ? -dev*s : dev*(s-1)))
// s (su) is the carrier sample index after Carrier::next at the symbol's first sample.
struct ScanK {
    int kind;
    float shift, freq, max;
    int map;
    __device__ static ScanK of(const TxParams& p) { return ScanK{p.ph_kind, p.ph_shift, p.ph_freq, p.ph_max, p.ph_map}; }
};
template <int KIND>
__device__ __forceinline__ float2 scan_step(const ScanK& k, float2 st, uint32_t idx, uint64_t su) {
#pragma clang fp contract(off)
    if (KIND == PH_DMPSK) {
        st.x = mod_trig_ieee(st.x + (float)idx * k.shift);
    } else if (KIND == PH_MFSK) {
        const float next = k.map ? (float)(2 * (int)idx) : (float)(2 * (int)idx - (int)k.max);
        st.y = st.y + (st.x - next) * k.freq * (float)su;
        st.y = mod_trig_ieee(st.y);
        st.x = next;
    } else {                                   // BFSK: st = (phase, prev bit)
        const float b = (float)(idx & 1u);
        if (b != st.y) {
            const float d = b == 1.0f ? -(k.freq * (float)su) : k.freq * (float)(su - 1u);
            st.x = mod_trig_ieee(st.x + d);
            st.y = b;
        }
    }
    return st;
}


// A bank of channels of one scanned kind (modem_tx_process_batch): one lane of wave 0 per channel
// (kScanCpw channels per workgroup) runs that channel's recurrence with scan_step — the same operations in
// the same order as tx_scan, so a channel's states are bit for bit those of its single call — while
// waves 1-3 stream the symbols through LDS: they decode block b + 1's symbol indices (each wave
// instruction one channel's 64 consecutive symbols, coalesced) and write block b - 1's states out,
// both double-buffered, one barrier per block. (The first form, one lane per channel loading its own
// symbols and storing its own states, touched 64 lines per memory instruction: 3 Msymbols/s per
// lane, profiles/r06_scan_rate.txt.) 16 channels per workgroup rather than 64: the three streaming
// waves, not the recurrences, bounded a 64-channel workgroup (a bank of 64 DMPSK channels 352 ->
// 1090 Msymbols/s, MFSK 351 -> 682, BFSK 400 -> 490; 8 per workgroup measured the same as 16).
// ps: the channels' parameter blocks in device memory.
// A single channel (tx_scan) runs the same body with one channel per workgroup: lane 0 of wave 0
// runs the recurrence while wave 1 streams (the earlier single form, every lane decoding 256
// indices, then lane 0 stepping, then every lane storing, serially: 6-9 Msymbols/s).
// scan_bank: channels ps[0 .. nc) (nc <= CPW) in this workgroup.
constexpr int kScanCpw = 16;
template <int KIND, int CPW>
__device__ __forceinline__ void scan_bank(const TxParams* __restrict__ ps, int nc) {
    constexpr int B = 64, S = B + 1;           // symbols per block; LDS row stride (conflict-free columns)
    __shared__ uint32_t sidx[2][CPW * S];
    __shared__ float2 sst[2][CPW * S];
    const int c0 = 0;
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6), lane = threadIdx.x & 63;
    int64_t nmax = 0;
    for (int c = 0; c < nc; ++c) nmax = ps[c0 + c].nsym > nmax ? ps[c0 + c].nsym : nmax;
    const int64_t nblk = (nmax + B - 1) / B;
    // waves 1-3: channel rows c = wave - 1, wave + 2, ... of block blk (issuing every row's loads
    // before the LDS writes measured no faster: 12.1 vs 11.2 ms for 64 x 2^16 DMPSK symbols)
    auto load_block = [&](int64_t blk) {
        for (int c = wave - 1; c < nc; c += 3) {
            const TxParams& q = ps[c0 + c];
            const int64_t m = blk * B + lane;
            sidx[blk & 1][c * S + lane] = m < q.nsym ? tx_symbol_index(q, m) : 0u;
        }
    };
    auto store_block = [&](int64_t blk) {
        for (int c = wave - 1; c < nc; c += 3) {
            const TxParams& q = ps[c0 + c];
            const int64_t m = blk * B + lane;
            if (m < q.nsym) q.scan[m] = sst[blk & 1][c * S + lane];
        }
    };
    float2 st = make_float2(0.f, 0.f);
    ScanK k{};
    int64_t nsym = 0;
    uint64_t s0 = 0, sps = 0;
    if (wave == 0 && lane < nc) {
        const TxParams& q = ps[c0 + lane];
        st = q.hist[0];
        k = ScanK::of(q);
        nsym = q.nsym;
        s0 = q.s0;
        sps = (uint64_t)q.sps;
    }
    if (wave > 0) load_block(0);
    __syncthreads();
    for (int64_t blk = 0; blk < nblk; ++blk) {
        if (wave == 0) {
            if (lane < nc) {
                const uint32_t* ix = &sidx[blk & 1][lane * S];
                float2* so = &sst[blk & 1][lane * S];
                const int64_t mb = blk * B;
                const int cnt = nsym - mb < B ? (int)(nsym - mb) : B;   // (<= 0: this channel is done)
                for (int j0 = 0; j0 < cnt; j0 += 16) {
                    uint32_t v[16];                    // the next 16 indices read ahead of the steps
#pragma unroll
                    for (int i = 0; i < 16; ++i) v[i] = ix[j0 + i];
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        if (j0 + i < cnt) {
                            st = scan_step<KIND>(k, st, v[i], s0 + (uint64_t)(mb + j0 + i) * sps + 1u);
                            so[j0 + i] = st;
                        }
                    }
                }
            }
        } else {
            if (blk + 1 < nblk) load_block(blk + 1);
            if (blk > 0) store_block(blk - 1);
        }
        __syncthreads();
    }
    if (wave > 0 && nblk > 0) store_block(nblk - 1);
    if (wave == 0 && lane < nc) ps[c0 + lane].hist_new[0] = st;
}
template <int KIND>
__global__ __launch_bounds__(256) void tx_scan_batch(const TxParams* __restrict__ ps, int nch) {
    const int c0 = (int)blockIdx.x * kScanCpw;
    scan_bank<KIND, kScanCpw>(ps + c0, nch - c0 < kScanCpw ? nch - c0 : kScanCpw);
}
template <int KIND>
__global__ __launch_bounds__(256) void tx_scan(const TxParams p) {
    __shared__ TxParams sp;                    // the parameter block where the body's loads reach it
    if (threadIdx.x == 0) sp = p;
    __syncthreads();
    scan_bank<KIND, 1>(&sp, 1);
}

hipError_t launch_tx_scan_batch(const TxParams* dps, int nch, int kind, hipStream_t s) {
    if (nch < 1) return hipSuccess;
    const dim3 grid((unsigned)((nch + kScanCpw - 1) / kScanCpw)), block(256);
    switch (kind) {
    case PH_DMPSK: hipLaunchKernelGGL(tx_scan_batch<PH_DMPSK>, grid, block, 0, s, dps, nch); break;
    case PH_MFSK: hipLaunchKernelGGL(tx_scan_batch<PH_MFSK>, grid, block, 0, s, dps, nch); break;
    case PH_BFSK: hipLaunchKernelGGL(tx_scan_batch<PH_BFSK>, grid, block, 0, s, dps, nch); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
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

hipError_t launch_tx_phasor(const TxParams& p, int dtype, int out_mode, hipStream_t s, bool scanned) {
    const int64_t nsamp = p.nsym * p.sps;
    if (p.scan != nullptr && !scanned) {
        switch (p.ph_kind) {
        case PH_DMPSK: hipLaunchKernelGGL(tx_scan<PH_DMPSK>, dim3(1), dim3(256), 0, s, p); break;
        case PH_MFSK: hipLaunchKernelGGL(tx_scan<PH_MFSK>, dim3(1), dim3(256), 0, s, p); break;
        case PH_BFSK: hipLaunchKernelGGL(tx_scan<PH_BFSK>, dim3(1), dim3(256), 0, s, p); break;
        default: return hipErrorInvalidValue;
        }
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


// The matrix-core variants are instantiated in their own translation units (modem_txm_*.hip,
// one per output form: the sources compile in parallel); here only their dispatch.
hipError_t launch_tx_mfma_batch(const TxBatch& b, int sps, int nks, const void* bfrag, int dtype,
                                hipStream_t s) {
    if (b.nch < 1 || b.nch > kBatchMax) return hipErrorInvalidValue;
    return dtype == 1 ? txm_sel_batch<__half>(b, sps, nks, bfrag, s) : txm_sel_batch<float>(b, sps, nks, bfrag, s);
}

int tx_mfma_ksteps(int sps, int K) {
    if (sps != 2 && sps != 4 && sps != 8 && sps != 16) return 0;
    const int need = (16 / sps + K - 1 + 31) / 32;
    int best = 0;
#define TXK(S, N) if (sps == S && N >= need && (best == 0 || N < best)) best = N;
    MODEM_TXM_TABLE(TXK)
#undef TXK
    return best;
}

hipError_t launch_tx_mfma(const TxParams& p, int sps, int nks, const void* bfrag, int dtype, int out_mode,
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

