// rust-modem_amd/csrc/modem_internal.h — kernel parameter blocks and launchers shared by
// modem_kernels.hip (device code) and modem_capi.cpp (the C ABI). Not part of the ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>

namespace mk {

// The RX MFMA kernels walk a call's tiles in rounds from the top down (rx_mfma_body), so the
// last samples a TX launch wrote are the first the RX reads. The TX store policy relies on it
// (modem_capi.cpp tx_nt_below: a single-channel launch of <= 256 MiB keeps its second half
// cacheable); rx_mfma_body asserts it. Changing the RX walk means revisiting that policy.
constexpr bool kRxTilesTopDown = true;

// One TX launch: symbols [0, nsym) of this call -> samples [0, nsym*sps).
struct TxParams {
    const uint8_t* bits;     // this call's bits, one byte per bit (device)
    const uint8_t* carry;    // ncarry leftover bits of the previous call (device)
    uint8_t* carry_new;      // leftover bits after this call (other buffer)
    const float2* hist;      // K-1 complex symbol values preceding symbol 0 (device)
    float2* hist_new;        // K-1 values preceding the next call's symbol 0
    const float2* lut;       // 2^bps complex points (device)
    const float* taps;       // polyphase taps, taps[t*sps + p] = h[p + sps*t], K*sps floats
    const float* taps_q;     // Q-rail taps (the I taps delayed by the Q offset), or null: = taps
    void* out;               // f32 or f16 samples (layout per out_mode)
    int64_t nt_below;        // tx_mfma: full sub-tiles of call samples < nt_below store non-temporally
    uint64_t s0;             // carrier sample of output sample 0
    int64_t nsym;            // symbols this call emits
    int64_t nsym_valid;      // symbols < nsym_valid are data, the rest are zero (flush)
    int64_t nbits;           // bits in `bits`
    int32_t ncarry;          // bits in `carry`
    int32_t ncarry_new;      // bits to leave in `carry_new`
    int32_t update_carry;    // 0 during flush
    int32_t bps;
    int32_t sps;             // runtime samples/symbol (generic kernel)
    int32_t K;               // taps per polyphase branch = ceil(ntaps / sps)
    int32_t fast_bits;       // ncarry == 0, bps in {1,2,4,8}, bits aligned to bps bytes
    int32_t exact_idx;       // every carrier index of this call is < 2^53 (exact as f64)
    int32_t idx46;           // ... and < 2^46 (tx_mfma's exact f32 index split, emit_full)
    float w;                 // Freq::sample_freq()
    // tx_mfma (split-f16 FIR): LUT as (re_hi, re_lo, im_hi, im_lo) halves of lut * 2^lut_scale_exp,
    // B fragments hold taps * 2^tap_scale_exp; lead = symbols before this call, mod 16/sps.
    const void* lut_h;
    int32_t lut_scale_exp;
    int32_t tap_scale_exp;
    int32_t lead;
    // levels: every LUT component is an integer multiple of one scale s, folded into the taps;
    // lut_h then holds the exact f16 integer levels (lo halves zero) and a symbol value v of the
    // history maps to the level rint(v * level_inv), level_inv = 1/s.
    int32_t levels;
    float level_inv;
    // tx_phasor (sample-dependent phasors, sample-and-hold): kind (modem_phasor_kind), the
    // symbols emitted before this call (DCQPSK parity), amplitude, CPFSK frequency, MSK
    // samples per bit, Q offset (0 or sps/2). `lut` then holds the DCQPSK table
    // (even-count block, then odd-count block); `hist[0].x` the index of the symbol before
    // symbol 0 (the offset Q rail's bits).
    int32_t ph_kind;
    uint64_t sym0;
    float ph_amp;
    float ph_freq;
    int32_t ph_spb;
    int32_t q_off;
    // DMPSK / MFSK / BFSK: per-symbol states of this call (tx_scan writes, tx_phasor reads),
    // the DMPSK shift, the MFSK map and max symbol. The handle state (DMPSK phase; MFSK
    // cur_coef, phase_offset; BFSK phase, prev bit) is hist[0] -> hist_new[0].
    float2* scan;
    float ph_shift;
    int32_t ph_map;
    float ph_max;
};

// One RX launch: input samples [0, N) (stream indices n_start ..), outputs k_first ..
struct RxParams {
    const void* x;           // this chunk: N complex samples (f32x2 or f16x2)
    const void* hist;        // HL samples preceding x (same dtype); zeros before the stream
    void* hist_new;          // HL samples preceding the next chunk
    void* out_iq;            // decimated filter outputs (f32x2 or f16x2), may be null
    uint8_t* out_sym;        // decisions, may be null
    const float* taps;       // polyphase taps, taps[b*K + t] = h[b + decim*t], decim*K floats
    const float2* slut;      // NEAREST slicer LUT (device)
    int64_t N;
    int64_t n_start;         // stream index of x[0]
    uint64_t c0;             // carrier sample of stream index 0
    int64_t k_first;         // first kept instant: n = k*decim + D
    int64_t nout;            // kept instants in this call
    int32_t K;               // taps per polyphase branch
    int32_t L;               // ntaps (generic kernel)
    int32_t HL;              // history length = K*decim - 1
    int32_t D;               // decim_offset
    int32_t decim;           // runtime decimation (generic kernel)
    int32_t x_aligned16;     // x is 16-byte aligned (pair loads)
    int32_t exact_idx;
    int32_t slicer_kind;
    int32_t bps;
    int32_t bits_per_carrier;
    float inv_scale;
    float max_symbol;
    float w;
    int32_t tap_scale_exp;   // rx_mfma: tables hold h * 2^tap_scale_exp
    float phase_offset;      // PLL offset added to the carrier phase (demodulator.rs:50)
    int32_t idx46;           // every carrier index of this call is < 2^46 (rx_mfma's f32 index split)
    const int* ka_in;        // rx_mfma: staging exponent the previous call ended with (INT_MIN: none)
    int* ka_out;             // rx_mfma: the one this call ends with (written with its last tile)
};

struct FirParams {
    const float* x;
    const float* hist;       // L-1 samples preceding x
    float* hist_new;
    float* y;
    const float* taps;       // h[k], L floats
    int64_t N;
    int32_t L;
};

// Launchers return hipSuccess or the launch error. They pick a specialised kernel for the
// common samples-per-symbol values and a generic one otherwise.
hipError_t launch_tx(const TxParams& p, int sps, int dtype, int out_mode, hipStream_t s);
// Sample-dependent phasors (DCQPSK, CPFSK, MSK; DMPSK, MFSK, BFSK after a serial symbol-state
// scan), sample-and-hold: tx_scan + tx_phasor.
// scanned: the states are already in p.scan (a batch's tx_scan_batch ran), only tx_phasor runs.
hipError_t launch_tx_phasor(const TxParams& p, int dtype, int out_mode, hipStream_t s, bool scanned = false);
// The serial state scan of DMPSK / MFSK / BFSK for nch channels of one phasor kind at once, one
// lane per channel (dps: their TxParams in device memory, p.scan set).
hipError_t launch_tx_scan_batch(const TxParams* dps, int nch, int kind, hipStream_t s);
// TX FIR on the matrix cores (tx_mfma, split-f16 MFMA): 32-symbol k-steps for (sps, K), or 0
// when no variant fits; bfrag = per-lane B fragments [ksteps][hi, lo][64 lanes][8 halves].
int tx_mfma_ksteps(int sps, int K);
// Channel batches (modem_tx_process_batch / modem_rx_process_batch): up to kBatchMax
// independent handles of one configuration in one launch; the launcher sets g, the
// workgroups per channel (workgroup b serves channel b / g), rot and xc (xcd_chunk of g).
constexpr int kBatchMax = 8;
struct TxBatch { TxParams p[kBatchMax]; int32_t nch; int32_t g; int32_t rot; int32_t xc; };
struct RxBatch { RxParams p[kBatchMax]; int32_t nch; int32_t g; int32_t rot; int32_t xc; };
// The per-channel rotation of a batch launch's workgroups (a multiple of 8, so that every tile
// keeps its XCD slot: blocks b and b + 8 share an XCD); 0 when g is not a multiple of 8.
// MODEM_BATCH_ROT=0 in the environment turns it off (A/B).
inline int32_t batch_rot(int32_t g, int32_t nch) {
    static const bool on = [] { const char* e = std::getenv("MODEM_BATCH_ROT"); return !e || e[0] != '0'; }();
    return on && g % 8 == 0 && 8 * (nch - 1) < g ? 8 : 0;
}
// mixed-carrier I/Q output only (OUT_IQ_MIXED); dtype 0 f32, 1 f16
hipError_t launch_tx_mfma_batch(const TxBatch& b, int sps, int nks, const void* bfrag, int dtype, hipStream_t s);
// complex mix only (MIX_COMPLEX); in and out of one dtype
hipError_t launch_rx_mfma_batch(const RxBatch& b, int decim, int nks, const void* tables, int dtype, hipStream_t s);
hipError_t launch_tx_mfma(const TxParams& p, int sps, int nks, const void* bfrag, int dtype,
                          int out_mode, hipStream_t s);
// RX matched filter on the matrix cores (rx_mfma, split-f16 MFMA): 32-sample k-steps for
// (decim, ntaps), or 0 when no variant fits.
int rx_mfma_ksteps(int decim, int L);
// Its tap tables: rx_mfma_table_copies(decim) copies q of the reversed taps
// T[x] = h[W - 1 - x] * 2^tap_scale_exp (W = 32*nks), copy q holding T[y + q*gcd(decim, 8)],
// each as hi then lo f16 halves of rx_mfma_table_len(decim, nks) entries.
constexpr int rx_mfma_table_copies(int decim) {
    return 8 / (decim % 8 == 0 ? 8 : decim % 4 == 0 ? 4 : decim % 2 == 0 ? 2 : 1);
}
// Padded so that the 16 lanes of every ds_read_b128 lane group read distinct LDS bank quads
// across the NC copies (bank model of MI355X_MICROARCH.md §LDS, checked by tests/test_lds_banks.py):
// len % 64 == 32 halves when decim % 8 == 4, else 16.
constexpr int rx_mfma_table_len(int decim, int nks) {
    const int n = (32 * nks + 15 * decim + 8 + 7) & ~7;
    const int r = decim % 8 == 4 ? 32 : 16;
    return n + ((r - (n % 64)) % 64 + 64) % 64;
}
hipError_t launch_rx_mfma(const RxParams& p, int decim, int nks, const void* tables, int in_dtype,
                          int out_dtype, int mix, hipStream_t s);
hipError_t launch_rx(const RxParams& p, int decim, int in_dtype, int out_dtype, int mix,
                     hipStream_t s);
// One loopback period (TX into the sample buffer rp.x == tp.out, then RX over it, complex
// mix, in and out of one dtype) as one persistent launch (modem_chain.hip); hipErrorNotSupported
// when the filters or the call's geometry have no fused form (run the two launches then);
// *form = 1 (chain_mfma) or 2 (chain_small: one RX tile per workgroup, LDS hand-off).
hipError_t launch_chain_mfma(const TxParams& tp, int sps, int nks_t, const void* bfrag, const RxParams& rp,
                             int nks_r, const void* tables, int dtype, hipStream_t s, int* form);
// The matrix-core variants by element types, instantiated in their own translation units
// (modem_txm_*.hip: OM = OUT_IQ_MIXED / BASEBAND / REAL, OutT = float / __half; modem_rxm_*.hip:
// MIX = MIX_COMPLEX / MIX_REFERENCE_REAL, InT, OutT = float / __half) and dispatched from
// launch_tx_mfma* / launch_rx_mfma* (hipErrorInvalidValue: no variant for the shape).
template <int OM, typename OutT>
hipError_t txm_sel(const TxParams& p, int sps, int nks, const void* bfrag, hipStream_t s);
template <typename OutT>
hipError_t txm_sel_batch(const TxBatch& b, int sps, int nks, const void* bfrag, hipStream_t s);
template <typename InT, int MIX, typename OutT>
hipError_t rxm_sel(const RxParams& p, int decim, int nks, const void* tables, hipStream_t s);
template <typename T>
hipError_t rxm_sel_batch(const RxBatch& b, int decim, int nks, const void* tables, hipStream_t s);
hipError_t launch_fir(const FirParams& p, hipStream_t s);
hipError_t launch_phases(float w, uint64_t s0, size_t n, float* out, hipStream_t s);
hipError_t launch_prng_bits(uint64_t seed, uint8_t* out, size_t nbits, hipStream_t s);

// Largest tap count the kernels accept (LDS budget).
constexpr int kMaxTaps = 4096;
// Zero steps appended to the polyphase tap buffers (look-ahead loads of the next chunk).
constexpr int kTapPad = 16;

}  // namespace mk
