// rust-modem_amd/csrc/modem_rxm.h — the RX matrix-core kernels (rx_mfma, rx_mfma_batch) and their
// launchers for every filter shape of modem_variants.h. Each modem_rxm_*.hip instantiates
// rxm_sel / rxm_sel_batch for some element types, so that the variants compile in parallel;
// modem_rx.hip dispatches to them (declarations in modem_internal.h).
#pragma once
#include <cstdlib>
#include "modem_rx_mfma.h"
#include "modem_variants.h"

namespace mk {

template <int DEC, int NKS, typename InT, int MIX, typename OutT, int NWF, int EM, int KS>
__global__ __launch_bounds__(256 * KS) __attribute__((amdgpu_waves_per_eu(RxMfma<DEC, NKS, InT, MIX, OutT, NWF, KS>::WPE)))
void rx_mfma(const RxParams p, const _Float16* __restrict__ tables, int xc) {
    rx_mfma_body<DEC, NKS, InT, MIX, OutT, NWF, EM, KS>(p, tables, xcd_slot(blockIdx.x, xc), gridDim.x);
}

// A batch of independent channels of one configuration (modem_rx_process_batch): workgroup
// b serves channel b / g as its workgroup b % g of g.
template <int DEC, int NKS, typename InT, int MIX, typename OutT, int NWF, int EM, int KS>
__global__ __launch_bounds__(256 * KS) __attribute__((amdgpu_waves_per_eu(RxMfma<DEC, NKS, InT, MIX, OutT, NWF, KS>::WPE)))
void rx_mfma_batch(const RxBatch b, const _Float16* __restrict__ tables) {
    const int ch = (int)(blockIdx.x / (unsigned)b.g);
    // channel ch's workgroups rotated by ch * b.rot (batch_rot): its workgroup 0, which also takes
    // the channel's general-path tile and its partial last tile, lands on another CU than the
    // other channels' workgroup 0
    unsigned bid = blockIdx.x - (unsigned)ch * b.g + (unsigned)(ch * b.rot);
    bid = bid >= (unsigned)b.g ? bid - (unsigned)b.g : bid;
    bid = (unsigned)xcd_slot(bid, b.xc);    // the channel's XCD-chunked slot (b.g a multiple of 8 b.xc)
    const RxParams p = b.p[ch];     // one bulk copy: the body's uses read registers, not kernarg
    rx_mfma_body<DEC, NKS, InT, MIX, OutT, NWF, EM, KS>(p, tables, bid, b.g);
}

template <int DEC, int NKS, typename InT, int MIX, typename OutT, int NWF, int EM, int KS>
static hipError_t rxm_go_em(const RxParams& p, const void* tables, hipStream_t s) {
    using K = RxMfma<DEC, NKS, InT, MIX, OutT, NWF, KS>;
    const int64_t ntiles = (p.nout + (p.k_first & 15) + K::TS - 1) / K::TS;
    const void* k = reinterpret_cast<const void*>(&rx_mfma<DEC, NKS, InT, MIX, OutT, NWF, EM, KS>);
    const unsigned grid = persistent_grid(k, K::NT, K::LDS_BYTES, ntiles);
    hipLaunchKernelGGL((rx_mfma<DEC, NKS, InT, MIX, OutT, NWF, EM, KS>), dim3(grid), dim3(K::NT), K::LDS_BYTES, s, p,
                       static_cast<const _Float16*>(tables), xcd_chunk(grid));
    return hipGetLastError();
}

template <int DEC, int NKS, typename InT, int MIX, typename OutT, int NWF, int EM, int KS>
static hipError_t rxm_go_batch_em(RxBatch b, const void* tables, hipStream_t s) {
    using K = RxMfma<DEC, NKS, InT, MIX, OutT, NWF, KS>;
    int64_t ntiles = 0;
    for (int c = 0; c < b.nch; ++c) {
        const int64_t t = (b.p[c].nout + (b.p[c].k_first & 15) + K::TS - 1) / K::TS;
        ntiles = t > ntiles ? t : ntiles;
    }
    const void* k = reinterpret_cast<const void*>(&rx_mfma_batch<DEC, NKS, InT, MIX, OutT, NWF, EM, KS>);
    const int64_t cap = persistent_grid(k, K::NT, K::LDS_BYTES, INT64_MAX);
    int64_t g = cap / b.nch;
    g = g < 1 ? 1 : g > ntiles ? (ntiles > 0 ? ntiles : 1) : g;
    b.g = (int32_t)g;
    b.rot = batch_rot(b.g, b.nch);
    b.xc = xcd_chunk(b.g);
    hipLaunchKernelGGL((rx_mfma_batch<DEC, NKS, InT, MIX, OutT, NWF, EM, KS>), dim3((unsigned)(g * b.nch)),
                       dim3(K::NT), K::LDS_BYTES, s, b, static_cast<const _Float16*>(tables));
    return hipGetLastError();
}

// The K-split launch (RxMfma KS = 2) for the 1024-instant tiles of the configurations that
// have one; MODEM_RX_KSPLIT=0 runs them with KS = 1 (the same results: RxMfma::KSO).
static bool rx_ksplit() {
    static const bool on = [] { const char* e = std::getenv("MODEM_RX_KSPLIT"); return !e || std::atoi(e) != 0; }();
    return on;
}

// Dispatch on the epilogue (the specialised ones exist only where rx_mfma_em can pick them)
// and on the tile size.
template <int DEC, int NKS, typename InT, int MIX, typename OutT, bool BATCH, typename Arg>
static hipError_t rxm_em(const Arg& a, int em, bool small, const void* tables, hipStream_t s) {
    constexpr bool loop = std::is_same<InT, OutT>::value && MIX == MIX_COMPLEX;
    constexpr bool f32 = std::is_same<InT, float>::value;
    constexpr int KS = RxMfma<DEC, NKS, InT, MIX, OutT, 4>::KSO ? 2 : 1;
    auto go = [&](auto emc) {
        constexpr int E = decltype(emc)::value;
        const bool ks = KS > 1 && rx_ksplit();
        if constexpr (BATCH)
            return small ? rxm_go_batch_em<DEC, NKS, InT, MIX, OutT, 1, E, 1>(a, tables, s)
                 : ks    ? rxm_go_batch_em<DEC, NKS, InT, MIX, OutT, 4, E, KS>(a, tables, s)
                         : rxm_go_batch_em<DEC, NKS, InT, MIX, OutT, 4, E, 1>(a, tables, s);
        else
            return small ? rxm_go_em<DEC, NKS, InT, MIX, OutT, 1, E, 1>(a, tables, s)
                 : ks    ? rxm_go_em<DEC, NKS, InT, MIX, OutT, 4, E, KS>(a, tables, s)
                         : rxm_go_em<DEC, NKS, InT, MIX, OutT, 4, E, 1>(a, tables, s);
    };
    switch (em) {
    case RXE_IQSYM: return go(std::integral_constant<int, loop ? RXE_IQSYM : RXE_GEN>());
    case RXE_IQSYM | RXE_NEAREST: return go(std::integral_constant<int, loop && f32 ? (RXE_IQSYM | RXE_NEAREST) : RXE_GEN>());
    case RXE_IQ: return go(std::integral_constant<int, loop && f32 ? RXE_IQ : RXE_GEN>());
    case RXE_SYM: return go(std::integral_constant<int, loop && f32 ? RXE_SYM : RXE_GEN>());
    default: return go(std::integral_constant<int, RXE_GEN>());
    }
}

template <int DEC, int NKS, typename InT, int MIX, typename OutT>
static hipError_t rxm_go(const RxParams& p, const void* tables, hipStream_t s) {
    return rxm_em<DEC, NKS, InT, MIX, OutT, false>(p, rx_mfma_em<InT, MIX, OutT>(p), rx_small_tiles(p.nout),
                                                   tables, s);
}

template <int DEC, int NKS, typename InT, typename OutT>
static hipError_t rxm_go_batch(const RxBatch& b, const void* tables, hipStream_t s) {
    int em = rx_mfma_em<InT, MIX_COMPLEX, OutT>(b.p[0]);          // one epilogue for the batch
    int64_t ninst = 0;
    for (int c = 0; c < b.nch; ++c) {
        if (rx_mfma_em<InT, MIX_COMPLEX, OutT>(b.p[c]) != em) em = RXE_GEN;
        ninst += b.p[c].nout;
    }
    return rxm_em<DEC, NKS, InT, MIX_COMPLEX, OutT, true>(b, em, rx_small_tiles(ninst), tables, s);
}

template <typename InT, int MIX, typename OutT>
hipError_t rxm_sel(const RxParams& p, int decim, int nks, const void* tables, hipStream_t s) {
#define RXM(D, N) if (decim == D && nks == N) return rxm_go<D, N, InT, MIX, OutT>(p, tables, s);
    MODEM_RXM_TABLE(RXM)
#undef RXM
    return hipErrorInvalidValue;
}

template <typename T>
hipError_t rxm_sel_batch(const RxBatch& b, int decim, int nks, const void* tables, hipStream_t s) {
#define RXM(D, N) if (decim == D && nks == N) return rxm_go_batch<D, N, T, T>(b, tables, s);
    MODEM_RXM_TABLE(RXM)
#undef RXM
    return hipErrorInvalidValue;
}

}  // namespace mk
