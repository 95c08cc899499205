// rust-modem_amd/csrc/modem_txm.h — the TX matrix-core kernels (tx_mfma, tx_mfma_batch) and their
// launchers for every filter shape of modem_variants.h. Each modem_txm_*.hip instantiates
// txm_sel / txm_sel_batch for some output forms, so that the variants compile in parallel;
// modem_tx.hip dispatches to them (declarations in modem_internal.h).
#pragma once
#include "modem_tx_mfma.h"
#include "modem_variants.h"

namespace mk {

template <int SPS, int NKS, int OUT_MODE, typename OutT, int SUB>
__global__ __launch_bounds__(256) void tx_mfma(const TxParams p, const th8* __restrict__ bfrag, int xc) {
    tx_mfma_body<SPS, NKS, OUT_MODE, OutT, SUB>(p, bfrag, xcd_slot(blockIdx.x, xc), gridDim.x);
}

// A batch of independent channels of one configuration (modem_tx_process_batch): workgroup
// b serves channel b / g as its workgroup b % g of g.
template <int SPS, int NKS, int OUT_MODE, typename OutT, int SUB>
__global__ __launch_bounds__(256) void tx_mfma_batch(const TxBatch b, const th8* __restrict__ bfrag) {
    const int ch = (int)(blockIdx.x / (unsigned)b.g);
    // channel ch's workgroups rotated by ch * b.rot (batch_rot): its workgroup 0, which also takes
    // the channel's general-path tile and its partial last tile, lands on another CU than the
    // other channels' workgroup 0
    unsigned bid = blockIdx.x - (unsigned)ch * b.g + (unsigned)(ch * b.rot);
    bid = bid >= (unsigned)b.g ? bid - (unsigned)b.g : bid;
    bid = (unsigned)xcd_slot(bid, b.xc);    // the channel's XCD-chunked slot (b.g a multiple of 8 b.xc)
    const TxParams p = b.p[ch];     // one bulk copy: the body's uses read registers, not kernarg
    tx_mfma_body<SPS, NKS, OUT_MODE, OutT, SUB>(p, bfrag, bid, b.g);
}

template <int SPS, int NKS, int OM, typename OutT, int SUB>
static hipError_t txm_go_sub(const TxParams& p, const void* bfrag, hipStream_t s) {
    using K = TxMfma<SPS, NKS, OM, OutT, SUB>;
    const int64_t ntiles = (p.nsym + p.lead + K::TS - 1) / K::TS;
    const size_t lds = (size_t)K::PLANES * 2 + ((size_t)1 << p.bps) * 8;
    const void* k = reinterpret_cast<const void*>(&tx_mfma<SPS, NKS, OM, OutT, SUB>);
    const unsigned grid = persistent_grid(k, K::NT, lds, ntiles);
    hipLaunchKernelGGL((tx_mfma<SPS, NKS, OM, OutT, SUB>), dim3(grid), dim3(K::NT), lds, s, p,
                       static_cast<const th8*>(bfrag), xcd_chunk(grid));
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
    b.rot = batch_rot(b.g, b.nch);
    b.xc = xcd_chunk(b.g);
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

template <int OM, typename OutT>
hipError_t txm_sel(const TxParams& p, int sps, int nks, const void* bfrag, hipStream_t s) {
#define TXM(S, N) if (sps == S && nks == N) return txm_go<S, N, OM, OutT>(p, bfrag, s);
    MODEM_TXM_TABLE(TXM)
#undef TXM
    return hipErrorInvalidValue;
}

template <typename OutT>
hipError_t txm_sel_batch(const TxBatch& b, int sps, int nks, const void* bfrag, hipStream_t s) {
#define TXM(S, N) if (sps == S && nks == N) return txm_go_batch<S, N, OUT_IQ_MIXED, OutT>(b, bfrag, s);
    MODEM_TXM_TABLE(TXM)
#undef TXM
    return hipErrorInvalidValue;
}

}  // namespace mk
