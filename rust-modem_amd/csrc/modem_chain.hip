// rust-modem_amd/csrc/modem_chain.hip — one period of the loopback chain (modem_chain_run:
// modulator.rs:85-100 + fir.rs:18-34 into the sample buffer, then demodulator.rs:44-56 +
// fir.rs:18-34 + the slicer over it) as ONE persistent launch instead of the TX and RX launches.
//
// Workgroup b owns a contiguous range of RX tiles [r0, r1) and the TX tiles that hold their
// samples, [m r0, m r1) (m = RX tile samples / TX tile samples; the last workgroup also takes
// any TX tiles past the last RX tile). It runs its TX tiles (TxMfma::run), then its RX tiles
// top-down (RxMfma::run), reading only samples it wrote itself: an RX tile's window also
// reaches H samples back into the previous TX tile, so before its own TX tiles the workgroup
// recomputes the last xs = ceil(H / 256) 16x16 sub-tiles of TX tile m r0 - 1 and stores them
// — the same values the owner of that tile stores there (the TX result of a sample does not
// depend on the path or the tile that computes it). No data crosses workgroups, so no flag,
// fence or cache maintenance is needed: a wave's stores are visible to the other waves of its
// workgroup after its vmcnt drain and a barrier (one CU, one L1, one L2).
//
// What this removes per period: one launch and the TX grid's drain before the RX grid starts
// (each workgroup's RX starts when its own TX ends). That pays for small, latency-bound calls
// only (chain_go below). Results are identical to the two launches
// (tests/test_gpu_chain_fused.py).
#include "modem_tx_mfma.h"
#include "modem_rx_mfma.h"
#include <cstdlib>

namespace mk {

// Which fused form the current launch_chain_mfma call took (1: chain_mfma, 2: chain_small);
// set and read on the calling host thread only.
static thread_local int g_chain_form = 1;

struct ChainGeo {
    int64_t nrx;     // RX tiles of the call
    int64_t ntx;     // TX tiles of the call
    int32_t m;       // TX tiles per RX tile
    int32_t xs;      // sub-tiles of TX tile m r0 - 1 a workgroup recomputes (r0 > 0)
};

template <int SPS, int NKS_T, int NKS_R, typename T, int SUB, int EM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RxMfma<SPS, NKS_R, T, MIX_COMPLEX, T, SUB>::WPE)))
void chain_mfma(const TxParams tp, const th8* __restrict__ bfrag, const RxParams rp,
                const _Float16* __restrict__ tables, const ChainGeo g) {
    using TK = TxMfma<SPS, NKS_T, OUT_IQ_MIXED, T, SUB>;
    using RK = RxMfma<SPS, NKS_R, T, MIX_COMPLEX, T, SUB>;     // SUB filter waves: tile sizes match
    extern __shared__ __attribute__((aligned(16))) _Float16 lds_c[];
    const int64_t bid = blockIdx.x, nb = gridDim.x;
    const int64_t r0 = g.nrx * bid / nb, r1 = g.nrx * (bid + 1) / nb;
    const int64_t t0 = r0 * g.m, t1 = bid == nb - 1 ? g.ntx : r1 * g.m, ts = 1;
    const int xs = g.xs;
    // ---- TX: tiles [t0, t1), after the last xs sub-tiles of tile t0 - 1
    if (bid == 0) tx_state_update(tp);
    {
        _Float16* pl = lds_c;
        th4* lut_s = reinterpret_cast<th4*>(lds_c + TK::PLANES);
        th8 bh[NKS_T], bl[NKS_T];
        load_bfrag(bfrag, bh, bl);
        bool done = false;
        if (tp.fast_bits && tp.idx46 && TK::out_ok(tp)) {
            done = true;
            switch (tp.bps) {
            case 1: TK::template run<1>(tp, pl, lut_s, bh, bl, t0, t1, ts, xs); break;
            case 2: TK::template run<2>(tp, pl, lut_s, bh, bl, t0, t1, ts, xs); break;
            case 4: TK::template run<4>(tp, pl, lut_s, bh, bl, t0, t1, ts, xs); break;
            case 8: TK::template run<8>(tp, pl, lut_s, bh, bl, t0, t1, ts, xs); break;
            default: done = false;
            }
        }
        if (!done) TK::template run<0>(tp, pl, lut_s, bh, bl, t0, t1, ts, xs);
    }
    // every wave's sample stores done before any wave of the workgroup reads them back
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // the RX history for the next period: the call's last HL samples, written by this
    // workgroup (checked on the host)
    if (bid == nb - 1) rx_state_update<T>(rp);
    // ---- RX: tiles r1 - 1 down to r0 (the last written first)
    _Float16* pl = lds_c;
    _Float16* tbl = lds_c + RK::TBL_OFF;
    float* red = reinterpret_cast<float*>(tbl + RK::NC * 2 * RK::TB);
    const TileSeq sq{r1 - 1, -1, r1 - r0, g.nrx};
    RK::template run<EM>(rp, pl, tbl, tables, red, sq, bid);
}

// The small call with one RX tile per workgroup (C2: 1024 tiles of 256 instants): the TX tile
// and its tail sub-tiles are staged together (TxMfma::one_tile), every emitted sample is also
// kept in an LDS window, and the RX stages its tile from there (RxMfma::run<EM, true>) instead of
// draining the stores and reading them back from HBM; the RX tap tables and *ka_in are requested
// at the kernel's start. LDS (halves): [TX planes x2 + LUT | RX planes] overlaid, then the RX
// tables, the RX votes / maxima, then the sample window.
template <int SPS, int NKS_T, int NKS_R>
struct SmallLds {
    using TK = TxMfma<SPS, NKS_T, OUT_IQ_MIXED, float, 1>;
    using RK = RxMfma<SPS, NKS_R, float, MIX_COMPLEX, float, 1>;
    static constexpr int TXH = 2 * TK::PLANES + 256 * 4;                 // + the largest LUT
    static constexpr int A = ((TXH > RK::TBL_OFF ? TXH : RK::TBL_OFF) + 7) & ~7;
    static constexpr int TBL = A, RED = A + RK::NC * 2 * RK::TB, RAW = (RED + 16 + 7) & ~7;
    static size_t bytes(int raw_n) { return (size_t)(RAW + 4 * raw_n) * 2; }
};

template <int SPS, int NKS_T, int NKS_R, int EM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RxMfma<SPS, NKS_R, float, MIX_COMPLEX, float, 1>::WPE)))
void chain_small(const TxParams tp, const th8* __restrict__ bfrag, const RxParams rp,
                 const _Float16* __restrict__ tables, const ChainGeo g) {
    using L = SmallLds<SPS, NKS_T, NKS_R>;
    using TK = typename L::TK;
    using RK = typename L::RK;
    extern __shared__ __attribute__((aligned(16))) _Float16 lds_s[];
    const int64_t bid = blockIdx.x, nb = gridDim.x, t = bid;
    if (bid == 0) tx_state_update(tp);
    // the RX's tap tables and staging exponent, requested first
    constexpr int NTB = RK::K_TAB8 / 256 + (RK::K_TAB8 % 256 ? 1 : 0);
    h8 tv[NTB];
#pragma unroll
    for (int k = 0; k < NTB; ++k) {
        const int j = threadIdx.x + k * 256;
        if (j < RK::K_TAB8) tv[k] = reinterpret_cast<const h8*>(tables)[j];
    }
    const int kin = *rp.ka_in;
    float2* raw = reinterpret_cast<float2*>(lds_s + L::RAW);
    const int64_t rb = (t * TK::TS - tp.lead) * SPS - (int64_t)g.xs * (16 * TK::SB * SPS);
    const int rn = g.xs * (16 * TK::SB * SPS) + TK::TS * SPS;
    const RawOut ro{raw, rb, rn};
    {
        _Float16* pl = lds_s;
        _Float16* pl2 = lds_s + TK::PLANES;
        th4* lut_s = reinterpret_cast<th4*>(lds_s + 2 * TK::PLANES);
        th8 bh[NKS_T], bl[NKS_T];
        load_bfrag(bfrag, bh, bl);
        bool done = false;
        if (tp.fast_bits && tp.idx46 && TK::out_ok(tp)) {
            done = true;
            switch (tp.bps) {
            case 1: TK::template one_tile<1>(tp, pl, pl2, lut_s, bh, bl, t, g.xs, ro); break;
            case 2: TK::template one_tile<2>(tp, pl, pl2, lut_s, bh, bl, t, g.xs, ro); break;
            case 4: TK::template one_tile<4>(tp, pl, pl2, lut_s, bh, bl, t, g.xs, ro); break;
            case 8: TK::template one_tile<8>(tp, pl, pl2, lut_s, bh, bl, t, g.xs, ro); break;
            default: done = false;
            }
        }
        if (!done) TK::template one_tile<0>(tp, pl, pl2, lut_s, bh, bl, t, g.xs, ro);
        // TX tiles past the last RX tile (their samples only feed the RX history)
        if (bid == nb - 1 && g.ntx > g.nrx) TK::template run<0>(tp, pl, lut_s, bh, bl, g.nrx, g.ntx, 1, 0);
    }
    _Float16* tbl = lds_s + L::TBL;
#pragma unroll
    for (int k = 0; k < NTB; ++k) {
        const int j = threadIdx.x + k * 256;
        if (j < RK::K_TAB8) reinterpret_cast<h8*>(tbl)[j] = tv[k];
    }
    if (bid == nb - 1) {                       // the RX history reads HBM: this workgroup's stores first
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        rx_state_update<float>(rp);
    }
    const TileSeq sq{t, -1, 1, g.nrx};
    RK::template run<EM, true>(rp, lds_s, tbl, tables, reinterpret_cast<float*>(lds_s + L::RED), sq, bid,
                               RxHandoff{raw, rb, rn, kin});
}


// Launch geometry, or false when the call does not fit the fused form (the caller then runs
// the two launches): matching tile sizes (small or not on both sides), RX tiles of m whole
// TX tiles, every RX window inside [its TX tiles' start - 256 xs, their end), the RX history
// inside the last workgroup's samples.
template <int SPS, int NKS_T, int NKS_R, typename T, int SUB>
static bool chain_geo(const TxParams& tp, const RxParams& rp, int64_t grid, ChainGeo& g) {
    using TK = TxMfma<SPS, NKS_T, OUT_IQ_MIXED, T, SUB>;
    using RK = RxMfma<SPS, NKS_R, T, MIX_COMPLEX, T, SUB>;
    constexpr int64_t TXS = (int64_t)TK::TS * SPS, RXS = (int64_t)RK::TS * SPS;   // samples per tile
    constexpr int64_t SUBS = 16 * TK::SB * SPS;                                    // per sub-tile (256)
    if (RXS % TXS) return false;
    g.m = (int32_t)(RXS / TXS);
    const int64_t lead_rx = rp.k_first & 15;
    g.nrx = (rp.nout + lead_rx + RK::TS - 1) / RK::TS;
    g.ntx = (tp.nsym + tp.lead + TK::TS - 1) / TK::TS;
    if (g.nrx <= 0 || g.nrx * g.m > g.ntx || rp.N != tp.nsym * SPS) return false;
    const int64_t q0 = (rp.k_first - lead_rx) * SPS + rp.D + 15 * SPS - RK::W + 1 - rp.n_start;   // q_lo_of(0)
    const int64_t tx0 = -(int64_t)tp.lead * SPS;                                   // TX tile 0's first sample
    const int64_t H = tx0 - q0;                                                    // window samples before it
    g.xs = H > 0 ? (int32_t)((H + SUBS - 1) / SUBS) : 0;
    if (g.xs > 4 * TK::SUB || q0 + RK::NS > tx0 + RXS) return false;
    if (grid < 1 || grid > g.nrx) return false;
    const int64_t rl = g.nrx * (grid - 1) / grid;                                  // the last workgroup's first RX tile
    const int64_t own = tx0 + rl * RXS - (rl > 0 ? g.xs * SUBS : 0);               // its first written sample
    const int64_t first = rp.N - rp.HL > 0 ? rp.N - rp.HL : 0;                     // rx_state_update's first read of x
    return first >= own;
}

template <int SPS, int NKS_T, int NKS_R, typename T, int SUB, int EM>
static hipError_t chain_go_em(const TxParams& tp, const void* bfrag, const RxParams& rp, const void* tables,
                              hipStream_t s) {
    using TK = TxMfma<SPS, NKS_T, OUT_IQ_MIXED, T, SUB>;
    using RK = RxMfma<SPS, NKS_R, T, MIX_COMPLEX, T, SUB>;
    const size_t tx_lds = (size_t)TK::PLANES * 2 + ((size_t)1 << tp.bps) * 8;
    const size_t lds = tx_lds > RK::LDS_BYTES ? tx_lds : RK::LDS_BYTES;
    const void* k = reinterpret_cast<const void*>(&chain_mfma<SPS, NKS_T, NKS_R, T, SUB, EM>);
    const int64_t lead_rx = rp.k_first & 15;
    const int64_t nrx = (rp.nout + lead_rx + RK::TS - 1) / RK::TS;
    unsigned grid = persistent_grid(k, 256, lds, nrx);
    ChainGeo g{};
    if (!chain_geo<SPS, NKS_T, NKS_R, T, SUB>(tp, rp, grid, g)) return hipErrorNotSupported;
    hipLaunchKernelGGL((chain_mfma<SPS, NKS_T, NKS_R, T, SUB, EM>), dim3(grid), dim3(256), lds, s, tp,
                       static_cast<const th8*>(bfrag), rp, static_cast<const _Float16*>(tables), g);
    return hipGetLastError();
}


template <int SPS, int NKS_T, int NKS_R, int EM>
static hipError_t chain_small_go(const TxParams& tp, const void* bfrag, const RxParams& rp, const void* tables,
                                 hipStream_t s) {
    using L = SmallLds<SPS, NKS_T, NKS_R>;
    using RK = typename L::RK;
    const int64_t nrx = (rp.nout + (rp.k_first & 15) + RK::TS - 1) / RK::TS;
    ChainGeo g{};
    if (!chain_geo<SPS, NKS_T, NKS_R, float, 1>(tp, rp, nrx, g) || g.m != 1) return hipErrorNotSupported;
    const size_t lds = L::bytes(g.xs * (16 * L::TK::SB * SPS) + L::TK::TS * SPS);
    const void* k = reinterpret_cast<const void*>(&chain_small<SPS, NKS_T, NKS_R, EM>);
    if ((int64_t)persistent_grid(k, 256, lds, nrx) < nrx) return hipErrorNotSupported;   // one tile each, all resident
    hipLaunchKernelGGL((chain_small<SPS, NKS_T, NKS_R, EM>), dim3((unsigned)nrx), dim3(256), lds, s, tp,
                       static_cast<const th8*>(bfrag), rp, static_cast<const _Float16*>(tables), g);
    g_chain_form = 2;
    return hipGetLastError();
}

// Small calls only (both sides on their small tiles: one 16x16 sub-tile per wave), and the
// steady-state epilogues only (the general one stays on the two launches). Small calls are
// latency-bound and the fused launch saves a launch and the TX grid's drain (C2 chain 11.2 vs
// 12.0 us, +9.5 % on the bench line, profiles/r03_chain_fused.txt). At size (C3) it is slower:
// 60.2 vs 56.5 us, the TX part alone 29.2 vs 25.8 us (its tail sub-tiles 1.8 us, contiguous
// tile ranges instead of grid-strided ones 0.7) while the RX part gains nothing (30.8 vs
// 30.4): at size the two launches' boundary is already small next to the per-CU work.
template <int SPS, int NKS_T, int NKS_R, typename T>
static hipError_t chain_go(const TxParams& tp, const void* bfrag, const RxParams& rp, const void* tables,
                           hipStream_t s) {
    if (!tx_small_tiles(tp.nsym, 16 / SPS) || !rx_small_tiles(rp.nout)) return hipErrorNotSupported;
    constexpr bool f32 = std::is_same<T, float>::value;
    auto go = [&](auto emc) -> hipError_t {
        constexpr int E = decltype(emc)::value;
        if constexpr (f32) {                   // one RX tile per workgroup: the LDS hand-off form
            const hipError_t e = chain_small_go<SPS, NKS_T, NKS_R, E>(tp, bfrag, rp, tables, s);
            if (e != hipErrorNotSupported) return e;
        }
        return chain_go_em<SPS, NKS_T, NKS_R, T, 1, E>(tp, bfrag, rp, tables, s);
    };
    switch (rx_mfma_em<T, MIX_COMPLEX, T>(rp)) {
    case RXE_IQSYM: return go(std::integral_constant<int, RXE_IQSYM>());
    case RXE_IQSYM | RXE_NEAREST:
        if constexpr (f32) return go(std::integral_constant<int, RXE_IQSYM | RXE_NEAREST>());
        return hipErrorNotSupported;
    case RXE_IQ:
        if constexpr (f32) return go(std::integral_constant<int, RXE_IQ>());
        return hipErrorNotSupported;
    case RXE_SYM:
        if constexpr (f32) return go(std::integral_constant<int, RXE_SYM>());
        return hipErrorNotSupported;
    default: return hipErrorNotSupported;
    }
}


// (sps = decim, TX k-steps, RX k-steps): the BASELINE chains (C2/C4 QPSK 65 taps sps 4, C3
// 129 taps sps 4, C5 513 taps sps 8); other filters run as the two launches.
#define CHAIN_TABLE(X) X(4, 1, 4) X(4, 2, 6) X(8, 3, 20)

hipError_t launch_chain_mfma(const TxParams& tp, int sps, int nks_t, const void* bfrag, const RxParams& rp,
                             int nks_r, const void* tables, int dtype, hipStream_t s, int* form) {
    g_chain_form = 1;
    auto sel = [&](auto tv) -> hipError_t {
        using T = decltype(tv);
#define CHN(S, NT_, NR_) \
        if (sps == S && nks_t == NT_ && nks_r == NR_) return chain_go<S, NT_, NR_, T>(tp, bfrag, rp, tables, s);
        CHAIN_TABLE(CHN)
#undef CHN
        return hipErrorNotSupported;
    };
    const hipError_t e = dtype == 1 ? sel(__half()) : sel(float());
    if (form) *form = g_chain_form;
    return e;
}

}  // namespace mk
