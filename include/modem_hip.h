/*
 * include/modem_hip.h — C ABI of the MI355X (gfx950) modem sample-path backend.
 *
 * This is the drop-in boundary for the hot path of ramtej/rust-modem (`src/modem`):
 *   bits -> symbol index -> (I,Q) LUT -> zero-stuff + RRC pulse-shaping FIR -> carrier mix
 *   -> [HBM sample buffer] -> conjugate mix -> matched filter at the decimated instants
 *   -> hard decision.
 * Every entry point is plain C: pointers, sizes, enums; no HIP or torch types (streams are
 * passed as an opaque `void*` hipStream_t; NULL = the device's default stream), so a Rust
 * `extern "C"` block, cgo or ctypes can bind it directly.
 *
 * Which reference interface each entry replaces (paths relative to the reference crate):
 *   modem_freq_sample_freq   freq.rs:19-26           Freq::new(hz, sr).sample_freq()
 *   modem_rates_sps          rates.rs:12-18          Rates::new(br, sr).samples_per_symbol
 *   modem_carrier_phase      carrier.rs:17-26,       Carrier::inner(s) = mod_trig(w * s as f32)
 *                            util.rs:3-6
 *   modem_phasor_lut         digital/phasor.rs:1-12, the memoryless DigitalPhasor plugins
 *                            bpsk.rs, qpsk.rs, qam.rs, bask.rs, mpsk.rs, apsk.rs, oqpsk.rs
 *   modem_tx_*               modulator.rs:64-101     DigitalModulator::new(&mut Carrier,
 *                            (+ fir.rs:3-35 for the   Box<DigitalPhasor>, Box<Source>) +
 *                            pulse shaping)           Iterator<Item=IQSample>; IQSample::
 *                                                     modulate (modulator.rs:45-48)
 *   modem_rx_*               demodulator.rs:7-56     Demodulator::new(Carrier, S, Fn()->
 *                                                     FIRFilter) + Iterator<Item=(f32,f32)>
 *   modem_fir_*              fir.rs:3-35             FIRFilter::new(&[f32]) + add(f32)->f32
 *   modem_chain_*            modulator.rs:85-100 then  one period of the sample-buffer loop:
 *                            demodulator.rs:44-56      the DigitalModulator's samples of a bit
 *                                                      buffer, then the Demodulator over them
 *   modem_chain_batch_*      the same, per channel       one period of a bank of independent
 *                                                      channels (one modulator and one
 *                                                      demodulator per stream)
 *
 * Conventions
 *   - Every function returns modem_status (0 = OK, negative = error) and never aborts.
 *     Where the reference panics (assert!, unwrap, out-of-range), this ABI returns
 *     MODEM_ERR_INVALID_ARG instead.
 *   - Taps and LUTs are copied at create time; the caller may free them afterwards.
 *   - I/O buffers are caller-owned. `*_process` accepts device pointers (asynchronous on
 *     `stream`) or host pointers (staged through the handle's device buffers; the call then
 *     synchronises `stream` before returning so the host buffers are valid).
 *   - Streaming: consecutive `*_process` calls equal one long call (the handle carries the
 *     carrier sample counter, the FIR history, leftover bits and the decimation phase);
 *     `*_flush` drains the filter with zeros.
 *   - One handle = one device; a handle is not thread-safe (it mirrors `&mut self`);
 *     distinct handles may be driven from different host threads. Device buffers passed to
 *     a handle must live on that handle's device (another GPU's memory: INVALID_ARG).
 */
#ifndef MODEM_HIP_H
#define MODEM_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: modem_tx_desc.q_offset; 3: the channel-batch entry points; 4: modem_rx_desc.phase_offset
 * (the descriptor grew 8 bytes: 80 -> 88), modem_pll_lock, MODEM_DTYPE_I16 and
 * MODEM_MIX_REFERENCE_REAL_EXACT; 5: modem_chain_* (no layout change; modem_chain_fused
 * added later, additive); 6: modem_chain_batch_* (additive, no layout change). Layouts:
 * INTEGRATION.md. */
#define MODEM_HIP_ABI_VERSION 6

typedef enum {
    MODEM_OK = 0,
    MODEM_ERR_INVALID_ARG = -1,   /* the reference would panic (assert!/unwrap/index) */
    MODEM_ERR_UNSUPPORTED = -2,   /* outside what this backend implements */
    MODEM_ERR_HIP = -3,           /* a HIP runtime call failed */
    MODEM_ERR_NO_DEVICE = -4,     /* no gfx950 device / bad device ordinal */
    MODEM_ERR_CAPACITY = -5,      /* output buffer too small for the call */
    MODEM_ERR_ALLOC = -6          /* host or device allocation failed */
} modem_status;

/* I16: real-valued samples, one native-endian int16 per sample (what `demodulate` reads from
 * stdin, bin/util.rs:3-37); RX input only, with MODEM_MIX_REFERENCE_REAL_EXACT. */
typedef enum { MODEM_DTYPE_F32 = 0, MODEM_DTYPE_F16 = 1, MODEM_DTYPE_I16 = 2 } modem_dtype;

/* TX output: complex (i,q)*e^{j phase} (IQSample::modulate, modulator.rs:45-48); the
 * un-mixed baseband (what `modulate --iq` writes, modulate.rs:110-113); or only the real
 * part (what `modulate` writes by default, modulate.rs:128-133). */
typedef enum {
    MODEM_OUT_IQ_MIXED = 0,
    MODEM_OUT_IQ_BASEBAND = 1,
    MODEM_OUT_REAL = 2
} modem_out_mode;

/* RX mix: complex conjugate x*e^{-j phase} (loopback contract), or the reference's
 * real-input mix x.re*(cos, -sin) with the 2x gain (demodulator.rs:46,52-55). REAL_EXACT is
 * the latter with every f32 operation of the reference in its order: glibc's cosf / sinf
 * results (the libm Rust's f32::cos / sin call on x86-64 Linux), the products, and
 * FIRFilter::add's sequential fold (fir.rs:18-34) — outputs bit-identical to Demodulator's
 * (demodulator.rs:44-56). A VALU kernel: for the text front-end, not for throughput. */
typedef enum { MODEM_MIX_COMPLEX = 0, MODEM_MIX_REFERENCE_REAL = 1, MODEM_MIX_REFERENCE_REAL_EXACT = 2 } modem_mix;

typedef enum {
    MODEM_SLICER_NONE = 0,        /* no decisions */
    MODEM_SLICER_NEAREST = 1,     /* argmin |r - lut[s]|^2, lowest index on ties */
    MODEM_SLICER_QAM_AXIS = 2     /* per-axis round+clamp, for QAM at phase 0 */
} modem_slicer_kind;

/* ---- memoryless DigitalPhasor plugins (host-side LUT builders) -------------------------- */
typedef enum {
    MODEM_PHASOR_BPSK = 1,   /* BPSK::new(phase, amplitude)            bpsk.rs:10-15 */
    MODEM_PHASOR_QPSK = 2,   /* QPSK::new(phase, amplitude)            qpsk.rs:11-17 */
    MODEM_PHASOR_QAM = 3,    /* QAM::new(bits_per_symbol, phase, amp)  qam.rs:15-30 */
    MODEM_PHASOR_BASK = 4,   /* BASK::new(amplitude)                   bask.rs:8-12 */
    MODEM_PHASOR_MPSK = 5,   /* MPSK::new(bps, phase_offset, amp)      mpsk.rs:14-21 */
    MODEM_PHASOR_APSK = 6,   /* APSK::new(amplitude, bps, rings)       apsk.rs:25-33 */
    MODEM_PHASOR_OQPSK = 7,  /* OQPSK::new(amplitude) (symbol map only) oqpsk.rs:9-13 */
    /* Phasors whose (i, q) also depend on the symbol count or the sample index. They have no
     * LUT (modem_phasor_lut returns MODEM_ERR_UNSUPPORTED): pass the descriptor to
     * modem_tx_create as modem_tx_desc.phasor (sample-and-hold only, ntaps == 0). */
    MODEM_PHASOR_DCQPSK = 8, /* DCQPSK::new(amplitude)                 dcqpsk.rs:16-21 */
    MODEM_PHASOR_CPFSK = 10, /* CPFSK::new(bps, rates, amp, deviation) cpfsk.rs:15-25; freq =
                              * Freq::new(deviation * baud / 2, sr).sample_freq() */
    MODEM_PHASOR_MSK = 11,   /* MSK::new(amplitude, samples_per_symbol) msk.rs:13-21 */
    /* Phasors that carry a phase from symbol to symbol in f32 (update() at every symbol
     * tick): the symbol states are computed by an exact serial scan on the device, then
     * evaluated per sample; exact, but one stream scans at tens of Msymbols/s. */
    MODEM_PHASOR_DMPSK = 9,  /* DMPSK::new(bps, amplitude, phase, shift) dmpsk.rs:16-23 */
    MODEM_PHASOR_MFSK = 12,  /* MFSK::new(bps, deviation, amplitude, map) mfsk.rs:46-59;
                              * freq = deviation.sample_freq(), mfsk_map 1 = IncreaseMap */
    MODEM_PHASOR_BFSK = 13   /* BFSK::new(deviation, amplitude)        bfsk.rs:12-20; freq as MFSK */
} modem_phasor_kind;

typedef struct { uint8_t start, end; float radius, phase; } modem_ring; /* apsk.rs:60-82 */

typedef struct {
    int32_t kind;                /* modem_phasor_kind */
    uint32_t bits_per_symbol;    /* QAM/MPSK/APSK; implied for the others */
    float phase;                 /* BPSK/QPSK/QAM phase, MPSK phase_offset */
    float amplitude;
    uint32_t nrings;             /* APSK */
    const modem_ring* rings;     /* APSK */
    float freq;                  /* CPFSK: its sample frequency (cpfsk.rs:20-21); MFSK, BFSK:
                                  * the deviation's sample frequency */
    uint32_t samples_per_symbol; /* MSK: samples per symbol (even, msk.rs:14) */
    float shift;                 /* DMPSK: phase step per symbol value (dmpsk.rs:20); its
                                  * initial phase is `phase` */
    uint32_t mfsk_map;           /* MFSK: 0 = DefaultMap (2s - max), 1 = IncreaseMap (2s) */
} modem_phasor_desc;

/* Slicer description; fill it with modem_phasor_slicer() or by hand. */
typedef struct {
    int32_t kind;                /* modem_slicer_kind */
    uint32_t bits_per_symbol;
    const float* lut;            /* NEAREST: 2 * 2^bps floats (i,q), host memory */
    uint32_t bits_per_carrier;   /* QAM_AXIS */
    float inv_scale;             /* QAM_AXIS: 1 / QAM amplitude scale (qam.rs:28) */
    float max_symbol;            /* QAM_AXIS: 2^bits_per_carrier - 1 */
} modem_slicer_desc;

const char* modem_status_str(modem_status s);
int32_t modem_abi_version(void);

/* Freq::new(hz, sr).sample_freq() — freq.rs:19-26 (f32, bit-exact). */
float modem_freq_sample_freq(uint64_t hz, uint64_t sr);
/* Rates::new(br, sr).samples_per_symbol — rates.rs:12-18. br == 0 -> INVALID_ARG. */
modem_status modem_rates_sps(uint64_t br, uint64_t sr, uint64_t* sps);
/* Carrier phase of absolute sample n, bit-exact to carrier.rs:17-19 + util.rs:3-6. */
float modem_carrier_phase(float sample_freq, uint64_t n);
/* The same phase for n consecutive samples s0.. computed by the device code path the
 * kernels use (out: n floats, device pointer; asynchronous on stream). */
modem_status modem_carrier_phases(float sample_freq, uint64_t s0, size_t n, float* out,
                                  int device, void* stream);
/* Bits per symbol of a phasor (DigitalPhasor::bits_per_symbol, phasor.rs:2). */
modem_status modem_phasor_bits(const modem_phasor_desc* d, uint32_t* bps);
/* (I,Q) table of a memoryless phasor: lut[2s], lut[2s+1] = i(_, b), q(_, b) where b are
 * the bits of s MSB-first (bytes_to_bits, digital/util.rs:5-11). 2*2^bps floats. */
modem_status modem_phasor_lut(const modem_phasor_desc* d, float* lut);
/* Pick the cheapest exact slicer for a phasor: QAM_AXIS for QAM at phase 0, else NEAREST
 * (lut must then stay valid until the RX handle is created). */
modem_status modem_phasor_slicer(const modem_phasor_desc* d, const float* lut,
                                 modem_slicer_desc* out);
/* Root-raised-cosine taps (GLUE, absent from the reference): centred at (L-1)/2,
 * roll-off beta, unit energy. */
modem_status modem_rrc_taps(uint32_t ntaps, uint32_t sps, double beta, float* out);

/* ---- TX: DigitalModulator + pulse shaping ------------------------------------------------ */
typedef struct modem_tx modem_tx;
typedef struct {
    uint32_t bits_per_symbol;    /* 1..8 */
    const float* lut;            /* 2 * 2^bps floats from modem_phasor_lut (host memory);
                                  * unused when `phasor` is set */
    uint32_t samples_per_symbol; /* Rates::samples_per_symbol, >= 1 */
    const float* taps;           /* pulse-shaping FIR (host memory) */
    uint32_t ntaps;              /* 0 = the reference's sample-and-hold (no FIR) */
    float sample_freq;           /* Freq::sample_freq() of the carrier */
    uint64_t s0;                 /* Carrier.sample at the first output sample */
    int32_t dtype;               /* modem_dtype of the output samples */
    int32_t out_mode;            /* modem_out_mode */
    uint32_t q_offset;           /* 0: Bits source. samples_per_symbol / 2: EvenOddOffset(Bits)
                                  * (data.rs:81-123, what modulate uses for oqpsk, modulate.rs:101-107):
                                  * Q changes half a symbol after I, and before the first Q tick
                                  * the phasor sees bit 0 (data.rs:84 `cur: [0, 0]`). Requires
                                  * bits_per_symbol == 2 and an even samples_per_symbol
                                  * (data.rs:91-92 asserts). With taps, the Q impulses sit at the
                                  * Q ticks (GLUE). */
    const modem_phasor_desc* phasor; /* NULL, or a DCQPSK / CPFSK / MSK phasor evaluated per
                                  * sample as DigitalModulator does (modulator.rs:85-100: the
                                  * symbol count since the stream start, and the carrier sample
                                  * index after Carrier::next); copied at create. */
} modem_tx_desc;

modem_status modem_tx_create(const modem_tx_desc* d, int device, modem_tx** out);
/* Consume `nbits` bits (one byte per bit, values 0/1 — data.rs:36) and write
 * floor((carry + nbits) / bps) * sps samples (2 values per sample for IQ modes, 1 for
 * OUT_REAL, each f32 or f16). Leftover bits (< bps) carry into the next call.
 * `cap` is in samples. */
modem_status modem_tx_process(modem_tx* h, const uint8_t* bits, size_t nbits, void* out,
                              size_t cap, size_t* produced, void* stream);
/* Several independent channels (distinct handles) in one call: the same results and handle
 * states as modem_tx_process(hs[c], bits[c], nbits[c], outs[c], caps[c], &produced[c], stream)
 * for c = 0 .. nch-1 in order. When every handle has the same matrix-core configuration
 * (sps, taps, bits per symbol, mixed I/Q output of one dtype, device) and every buffer is
 * device memory, up to 8 channels share one kernel launch. When every handle has the same
 * scanned phasor kind (DMPSK, MFSK, BFSK: a serial f32 state recurrence per stream,
 * dmpsk.rs:29-33, mfsk.rs:68-75, bfsk.rs:42-53) and every buffer is device memory, the
 * channels' state scans run as one launch, one lane per channel, each bit for bit its single
 * call's. Otherwise the calls run one by one.
 * No reference counterpart (the reference drives one DigitalModulator per stream,
 * modulator.rs:64-101): the multi-channel form of that loop, SURVEY.md §8e. */
modem_status modem_tx_process_batch(modem_tx* const* hs, size_t nch, const uint8_t* const* bits,
                                    const size_t* nbits, void* const* outs, const size_t* caps,
                                    size_t* produced, void* stream);
/* Append ceil((ntaps-1)/sps) all-zero symbols so the FIR tail drains. */
modem_status modem_tx_flush(modem_tx* h, void* out, size_t cap, size_t* produced, void* stream);
/* Samples that the next call will start at (Carrier.sample, carrier.rs:6). */
uint64_t modem_tx_sample(const modem_tx* h);
modem_status modem_tx_destroy(modem_tx* h);

/* ---- RX: Demodulator + matched filter + decimation + slicer ----------------------------- */
typedef struct modem_rx modem_rx;
typedef struct {
    float sample_freq;           /* carrier (demodulator.rs:20) */
    uint64_t s0;                 /* Carrier.sample of the first input sample */
    const float* taps;           /* matched filter / lowpass (host memory) */
    uint32_t ntaps;              /* >= 1 */
    uint32_t decim;              /* keep every decim-th filter output; 1 = full rate */
    uint32_t decim_offset;       /* keep outputs n = k*decim + decim_offset (stream index) */
    int32_t mix;                 /* modem_mix */
    int32_t in_dtype;            /* modem_dtype of the input I/Q samples */
    int32_t out_dtype;           /* modem_dtype of the decimated I/Q output */
    modem_slicer_desc slicer;    /* decisions (kind NONE for none) */
    float phase_offset;          /* PLL::phase_offset added to every carrier phase
                                  * (demodulator.rs:50); 0 = unlocked. See modem_pll_lock. */
} modem_rx_desc;

modem_status modem_rx_create(const modem_rx_desc* d, int device, modem_rx** out);
/* Consume n complex input samples (interleaved i,q); write the decimated filter outputs
 * (interleaved i,q; may be NULL) and u8 decisions (may be NULL) for every kept instant in
 * this chunk. `cap` is in symbols. */
modem_status modem_rx_process(modem_rx* h, const void* in, size_t n, void* out_iq,
                              uint8_t* out_sym, size_t cap, size_t* produced, void* stream);
/* Several channels in one call, as modem_rx_process on each handle in order (out_iq[c] and
 * out_sym[c] may be NULL). Fused into one launch per 8 channels when every handle has the
 * same matrix-core configuration (decimation, taps, complex mix, one I/Q dtype in and out,
 * device) and every buffer is device memory. The multi-channel form of Demodulator::next
 * (demodulator.rs:44-56), SURVEY.md §8e. */
modem_status modem_rx_process_batch(modem_rx* const* hs, size_t nch, const void* const* ins, const size_t* ns,
                                    void* const* out_iq, uint8_t* const* out_sym, const size_t* caps,
                                    size_t* produced, void* stream);
/* Feed ntaps-1 zero samples (drains the matched filter). */
modem_status modem_rx_flush(modem_rx* h, void* out_iq, uint8_t* out_sym, size_t cap,
                            size_t* produced, void* stream);
uint64_t modem_rx_sample(const modem_rx* h);
modem_status modem_rx_destroy(modem_rx* h);

/* ---- One TX -> RX period over fixed device buffers ------------------------------------- */
/* A prepared step of the sample-buffer loop: modem_chain_run(c) equals
 *   modem_tx_process(tx, bits, nbits, samples, cap, &n, stream);
 *   modem_rx_process(rx, samples, n, out_iq, out_sym, out_cap, &k, stream);
 * (produced = n, produced_out = k), with the buffers checked once by modem_chain_create:
 * device memory of the handles' one device (else INVALID_ARG); the TX writes interleaved
 * complex samples (MODEM_OUT_IQ_MIXED or BASEBAND) of the RX's in_dtype. The handles stay
 * usable on their own; the plan keeps pointers to them and to the buffers (destroy it first). */
typedef struct modem_chain modem_chain;
modem_status modem_chain_create(modem_tx* tx, modem_rx* rx, const uint8_t* bits, size_t nbits,
                                void* samples, size_t cap, void* out_iq, uint8_t* out_sym,
                                size_t out_cap, modem_chain** out);
modem_status modem_chain_run(modem_chain* c, size_t* produced, size_t* produced_out, void* stream);
/* How the last modem_chain_run ran: 1 or 2 = one launch (the TX and RX of the period fused:
 * small calls with the common filters, tile geometry permitting; 2 = the form with one RX tile
 * per workgroup that hands the samples over in LDS; results identical either way), 0 = the two
 * launches, -1 = no run yet or c == NULL. MODEM_CHAIN_FUSED=0 in the environment at create time
 * forces 0. */
int modem_chain_fused(const modem_chain* c);
modem_status modem_chain_destroy(modem_chain* c);

/* A prepared step of a channel bank (independent channel streams, BASELINE
 * config 4): modem_chain_batch_run(c) equals, for every channel i < nch,
 *   modem_tx_process(txs[i], bits[i], nbits[i], samples[i], caps[i], &n[i], stream);
 *   modem_rx_process(rxs[i], samples[i], n[i], out_iq[i], out_sym[i], out_caps[i], &k[i], stream);
 * run as one TX launch and then one RX launch per `group` consecutive channels (1 <= group <= 8;
 * a group of at most 192 MiB of samples is re-read from the Infinity Cache, a larger one — C4's
 * default 8 x 32 MiB — is stored non-temporally and re-read from HBM, which measured faster
 * for it, profiles/r05_c4_policy.txt). modem_chain_batch_create
 * checks the buffers (device memory of the handles' one device) and the handles (one matrix-core
 * configuration for all TX and one for all RX handles, distinct handles, RX in_dtype = TX dtype,
 * complex mix, interleaved complex TX output) once: INVALID_ARG / UNSUPPORTED otherwise, nothing
 * created. produced / produced_out (nch entries each, may be NULL) receive n[i] and k[i].
 * With more than one group the groups alternate between `stream` and a stream of the plan's
 * own (joined to `stream` by events at the start and end of every run), so that one group's RX
 * overlaps the next group's TX; the run is asynchronous on `stream` as a whole.
 * MODEM_CHAIN_BATCH_LANES=1 in the environment at create time keeps every launch on `stream`.
 * Errors: CAPACITY (checked for every channel before any launch) leaves every handle untouched;
 * a launch error (HIP) part-way through a run leaves the groups before it advanced and the
 * rest not, so the plan is marked failed and every later run returns MODEM_ERR_HIP (destroy
 * it; its handles' streams no longer line up). The caller's stream is still joined to the
 * plan's own (best effort) so that it stays ordered after the launches already queued. */
typedef struct modem_chain_batch modem_chain_batch;
modem_status modem_chain_batch_create(modem_tx* const* txs, modem_rx* const* rxs, size_t nch, size_t group,
                                      const uint8_t* const* bits, const size_t* nbits, void* const* samples,
                                      const size_t* caps, void* const* out_iq, uint8_t* const* out_sym,
                                      const size_t* out_caps, modem_chain_batch** out);
modem_status modem_chain_batch_run(modem_chain_batch* c, size_t* produced, size_t* produced_out, void* stream);
modem_status modem_chain_batch_destroy(modem_chain_batch* c);

/* Demodulator::lock_phase (demodulator.rs:32-36): PLL::handle (pll.rs:16-22) over the n
 * complex samples x_iq (host memory; the reference uses n = 64), with the carrier phases of
 * samples s0 .. s0+n-1, starting from *phase_offset (0 for a new PLL). Control logic over a
 * few serial samples: evaluated on the host with the reference's f32 operations. */
modem_status modem_pll_lock(float sample_freq, uint64_t s0, const float* x_iq, size_t n,
                            float* phase_offset);

/* ---- FIRFilter: real-valued causal FIR over a stream (fir.rs:3-35) ---------------------- */
typedef struct modem_fir modem_fir;
modem_status modem_fir_create(const float* taps, uint32_t ntaps, int device, modem_fir** out);
/* out[i] = FIRFilter::add(in[i]) for consecutive samples (f32, same count in and out),
 * bit-identical: the reference's fold order, separate multiply and add. */
modem_status modem_fir_process(modem_fir* h, const float* in, float* out, size_t n, void* stream);
modem_status modem_fir_destroy(modem_fir* h);

/* ---- synthetic input (GLUE): splitmix64 bit stream, one byte per bit ------------------- */
/* bit i = (word[i/64] >> (i%64)) & 1, word j = splitmix64 output j+1 from `seed`.
 * `out` must be a device pointer. */
modem_status modem_prng_bits(uint64_t seed, uint8_t* out, size_t nbits, int device, void* stream);

#ifdef __cplusplus
}
#endif
#endif
