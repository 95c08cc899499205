/*
 * oracle/modem_oracle.h — TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * A plain-C restatement of the sample hot path of ramtej/rust-modem (`src/modem`), one
 * function per reference item, each citing the reference file:line it follows
 * (paths relative to the reference crate root). Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library (oracle/_build/libmodem_oracle.so).
 *
 * Numerics: compiled with -O2 -ffp-contract=off and no fast-math, so every f32 operation is
 * rounded exactly as rustc (which never fuses a*b+c) rounds it; Rust's f32 sin/cos/floor/
 * sqrt/atan2 lower to the same glibc libm calls used here.
 *
 * Pinning: the reference's own known-answer tests (data.rs:194-279, digital/util.rs:21-33,
 * qam.rs:68-84, mpsk.rs:49-63, dmpsk.rs:50-84) are replayed against this library in
 * tests/test_oracle_kat.py. FIRFilter, Carrier, IQSample::modulate and Demodulator have no
 * reference test: they are cross-checked against an independent numpy restatement
 * (tests/test_oracle_crosscheck.py). Items marked GLUE do not exist in the reference
 * (zero-stuffing, RRC taps, decimation, slicer, PRNG): parity for them is build-defined.
 */
#ifndef MODEM_ORACLE_H
#define MODEM_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- util.rs / digital/util.rs ------------------------------------------------------- */
float    or_mod_trig(float x);                                  /* util.rs:3-6 */
float    or_bit_to_sign(uint8_t b);                             /* digital/util.rs:1-3 */
uint8_t  or_bytes_to_bits(const uint8_t* bytes, size_t len);    /* digital/util.rs:5-11 */
size_t   or_max_symbol(size_t bits_per_symbol);                 /* digital/util.rs:13-15 */

/* ---- freq.rs / carrier.rs / rates.rs -------------------------------------------------- */
float    or_freq_ang_freq(size_t hz);                           /* freq.rs:19-21 */
float    or_freq_sample_freq(size_t hz, size_t sr);             /* freq.rs:24-26 */
size_t   or_rates_samples_per_symbol(size_t br, size_t sr);     /* rates.rs:12-18 */

typedef struct { float sample_freq; uint64_t sample; } or_carrier;   /* carrier.rs:4-7 */
void     or_carrier_init(or_carrier* c, float sample_freq, uint64_t sample); /* carrier.rs:10-15 */
float    or_carrier_inner(const or_carrier* c, uint64_t s);    /* carrier.rs:17-19 */
float    or_carrier_next(or_carrier* c);                       /* carrier.rs:21-26 */
/* Vector form for tests: phase of absolute samples s0 .. s0+n-1. */
void     or_carrier_phases(float sample_freq, uint64_t s0, size_t n, float* out);

/* ---- data.rs ---------------------------------------------------------------------------- */
enum { OR_CHANGED = 0, OR_UNCHANGED = 1, OR_FINISHED = 2 };    /* data.rs:3-8 */

typedef struct { size_t samples_per_symbol, counter; } or_symbol_clock;   /* data.rs:14-17 */
void     or_symbol_clock_init(or_symbol_clock* c, size_t sps); /* data.rs:20-25 */
int      or_symbol_clock_next(or_symbol_clock* c);             /* data.rs:27-32 */

typedef struct {                                                /* data.rs:35-40 */
    const uint8_t* bits; size_t nbits;
    or_symbol_clock clock; size_t bits_per_symbol, idx;
} or_bits_source;
void     or_bits_init(or_bits_source* s, const uint8_t* bits, size_t nbits,
                      size_t sps, size_t bps);                  /* data.rs:43-52 */
/* returns OR_CHANGED / OR_UNCHANGED / OR_FINISHED; *slice points at bps bits */
int      or_bits_next(or_bits_source* s, const uint8_t** slice); /* data.rs:66-78 */

typedef struct {                                                /* data.rs:125-129 */
    const char* text; size_t len, pos;
    or_symbol_clock clock; uint8_t bits[8]; size_t nbits;
    int panicked;                  /* set where data.rs:155 assert! would panic */
} or_ascii_bits;
void     or_ascii_init(or_ascii_bits* a, const char* text, size_t len, size_t sps, size_t bps);
int      or_ascii_read_bits(or_ascii_bits* a);                  /* data.rs:161-171 */
int      or_ascii_next(or_ascii_bits* a, const uint8_t** slice); /* data.rs:174-185 */

/* `Box<Source>`: the two sources the CLI builds (modulate.rs:98-107). */
typedef struct { int is_ascii; or_bits_source bits; or_ascii_bits ascii; } or_source;
int      or_source_next(or_source* s, const uint8_t** slice);   /* data.rs:10-12 */

typedef struct {                                                /* data.rs:81-85 */
    or_source data; or_symbol_clock clock; uint8_t cur[2];
} or_even_odd;
/* data.rs:88-99; returns -1 where the asserts at :91-92 fail. `inner` is copied. */
int      or_even_odd_init(or_even_odd* e, const or_source* inner, size_t sps, size_t bps);
int      or_even_odd_next(or_even_odd* e, const uint8_t** slice); /* data.rs:102-122 */

/* ---- digital/<x>.rs : DigitalPhasor plugins ---------------------------------------------- */
enum {
    OR_BPSK = 1, OR_QPSK = 2, OR_QAM = 3, OR_BASK = 4, OR_MPSK = 5, OR_APSK = 6,
    OR_OQPSK = 7, OR_DCQPSK = 8, OR_DMPSK = 9, OR_CPFSK = 10, OR_MSK = 11, OR_MFSK = 12, OR_BFSK = 13,
};
typedef struct { uint8_t start, end; float radius, phase; } or_ring;       /* apsk.rs:60-67 */
typedef struct {
    int kind;
    size_t bits_per_symbol, bits_per_carrier;
    float amplitude, phase, phase_cos, phase_sin, max_symbol, num_symbols, shift;
    int even;                      /* dcqpsk.rs:12 */
    int nrings; or_ring rings[8];  /* apsk.rs:18 */
    float freq;                    /* cpfsk.rs:10; mfsk.rs:39 / bfsk.rs:6 deviation */
    size_t samples_per_bit;        /* msk.rs:8 */
    float cur_coef;                /* mfsk.rs:43 */
    int increase_map;              /* mfsk.rs: IncreaseMap (1) or DefaultMap (0) */
    uint8_t prev;                  /* bfsk.rs:9 */
} or_phasor;
/* Constructors mirror the reference `new` functions; return 0 on success, -1 on the
 * reference's assert! failure. */
int  or_bpsk_new(or_phasor* p, float phase, float amplitude);             /* bpsk.rs:10-15 */
int  or_qpsk_new(or_phasor* p, float phase, float amplitude);             /* qpsk.rs:11-17 */
int  or_qam_new(or_phasor* p, size_t bps, float phase, float amplitude);  /* qam.rs:15-30 */
int  or_bask_new(or_phasor* p, float amplitude);                          /* bask.rs:8-12 */
int  or_mpsk_new(or_phasor* p, size_t bps, float phase_offset, float amplitude); /* mpsk.rs:14-21 */
int  or_apsk_new(or_phasor* p, float amplitude, size_t bps,
                 const or_ring* rings, int nrings);                       /* apsk.rs:25-33 */
int  or_oqpsk_new(or_phasor* p, float amplitude);                         /* oqpsk.rs:9-13 */
int  or_dcqpsk_new(or_phasor* p, float amplitude);                        /* dcqpsk.rs:16-21 */
int  or_dmpsk_new(or_phasor* p, size_t bps, float amplitude, float phase, float shift); /* dmpsk.rs:16-23 */
/* CPFSK::new(bps, Rates::new(br, sr), amplitude, deviation)                   cpfsk.rs:15-25 */
int  or_cpfsk_new(or_phasor* p, size_t bps, size_t br, size_t sr, float amplitude, size_t deviation);
int  or_msk_new(or_phasor* p, float amplitude, size_t samples_per_symbol);        /* msk.rs:13-21 */
/* MFSK::new(bps, deviation.sample_freq(), amplitude, map)                       mfsk.rs:46-59 */
int  or_mfsk_new(or_phasor* p, size_t bps, float deviation, float amplitude, int increase_map);
int  or_bfsk_new(or_phasor* p, float deviation, float amplitude);                 /* bfsk.rs:12-20 */
size_t or_phasor_bits_per_symbol(const or_phasor* p);                     /* phasor.rs:2 */
void   or_phasor_update(or_phasor* p, uint64_t s, const uint8_t* b, size_t len); /* phasor.rs:4 */
float  or_phasor_i(const or_phasor* p, uint64_t s, const uint8_t* b, size_t len); /* phasor.rs:6 */
float  or_phasor_q(const or_phasor* p, uint64_t s, const uint8_t* b, size_t len); /* phasor.rs:7 */

/* ---- fir.rs ------------------------------------------------------------------------------ */
typedef struct { const float* coefs; size_t len; float* history; size_t idx; } or_fir; /* fir.rs:3-7 */
int   or_fir_init(or_fir* f, const float* coefs, size_t len);   /* fir.rs:10-16 (allocates) */
void  or_fir_free(or_fir* f);
float or_fir_calc(const or_fir* f);                              /* fir.rs:18-25 */
float or_fir_add(or_fir* f, float sample);                       /* fir.rs:27-34 */
/* Block form: out[i] = FIRFilter::add(in[i]) for a fresh filter. */
void  or_fir_block(const float* coefs, size_t len, const float* in, size_t n, float* out);

/* ---- modulator.rs ------------------------------------------------------------------------ */
typedef struct { float carrier, i, q; } or_iq_sample;            /* modulator.rs:22-26 */
float or_iq_real(const or_iq_sample* s, float cos_, float sin_); /* modulator.rs:37-39 */
float or_iq_imag(const or_iq_sample* s, float cos_, float sin_); /* modulator.rs:41-43 */
void  or_iq_modulate(const or_iq_sample* s, float* re, float* im); /* modulator.rs:45-48 */

/* DigitalModulator over a Bits source (modulator.rs:64-101). Returns samples written
 * (stops at Finished or cap). `changed`, if non-NULL, receives 1 on symbol ticks. */
size_t or_digital_modulate(or_carrier* c, or_phasor* p, const uint8_t* bits, size_t nbits,
                           size_t sps, or_iq_sample* out, uint8_t* changed, size_t cap);

/* ---- pll.rs / demodulator.rs ------------------------------------------------------------ */
typedef struct { float phase_offset; } or_pll;                   /* pll.rs:5-7 */
void  or_pll_handle(or_pll* p, float carrier_phase, float x_re, float x_im); /* pll.rs:16-22 */
/* Demodulator::next over a whole block, real input `x_re`, lock_phase skipped
 * (demodulator.rs:44-56). out_i/out_q are full-rate. */
void  or_demodulate(float sample_freq, uint64_t s0, float phase_offset,
                    const float* taps, size_t ntaps,
                    const float* x_re, size_t n, float* out_i, float* out_q);

/* demodulate.rs:29-43 with the filters as arguments (the binary hard-codes a 23-tap Hilbert and
 * a 64-tap low-pass, demodulate.rs:47-150): analytic = (x, hilbert.add(x)) per sample,
 * Demodulator::new(Carrier::new(freq), analytic, lowpass), lock_phase() (64 samples through the
 * PLL, demodulator.rs:32-36), then Demodulator::next for every remaining sample. Returns the
 * outputs written (n - 64; 0 if n < 64, where the reference's unwrap panics). */
size_t or_demodulate_front(float sample_freq, const float* x, size_t n, const float* hilbert, size_t nh,
                           const float* lowpass, size_t nlp, float* out_i, float* out_q, float* phase_offset);

/* ---- GLUE (absent from the reference; build-defined, parity unpinned by the reference) --- */
uint64_t or_splitmix64_next(uint64_t* state);
/* nbits bits, one byte per bit (data.rs:36 layout): bit i = (word[i/64] >> (i%64)) & 1 */
void  or_prng_bits(uint64_t seed, uint8_t* out, size_t nbits);
/* Root-raised-cosine taps, odd or even length, centred at (L-1)/2, unit energy. */
int   or_rrc_taps(size_t ntaps, size_t sps, double beta, float* out);
/* (I,Q) table: lut[2*s], lut[2*s+1] = phasor.i/q(0, bits of s MSB-first) (phasor.rs:9-11) */
int   or_phasor_lut(const or_phasor* p, float* lut);

enum { OR_SLICER_NEAREST = 0, OR_SLICER_QAM_AXIS = 1 };
typedef struct {
    int kind; size_t bps; const float* lut;     /* NEAREST */
    int bits_per_carrier; float inv_scale; float max_symbol;   /* QAM_AXIS */
} or_slicer;
uint8_t or_slice(const or_slicer* s, float re, float im);

enum { OR_MIX_COMPLEX = 0, OR_MIX_REFERENCE_REAL = 1 };
enum { OR_OUT_IQ_MIXED = 0, OR_OUT_IQ_BASEBAND = 1, OR_OUT_REAL = 2 };

/* TX chain, reference loop structure: DigitalModulator (timing + phase) -> zero-stuff
 * (GLUE) -> FIRFilter on I and on Q -> IQSample::modulate. ntaps == 0 keeps the reference
 * sample-and-hold (no FIR). flush_syms extra all-zero symbols are appended (carrier keeps
 * running). out holds 2 floats per sample (OUT_IQ_*) or 1 (OUT_REAL). Returns samples. */
size_t or_tx_chain(or_phasor* p, const uint8_t* bits, size_t nbits, size_t sps,
                   const float* taps, size_t ntaps, float sample_freq, uint64_t s0,
                   size_t flush_syms, int out_mode, float* out);

/* The same with the source chosen as the modulate CLI does (modulate.rs:101-107): even_odd
 * != 0 wraps the bits in EvenOddOffset (data.rs:81-123; bps == 2, sps even), so Q changes half
 * a symbol after I. With taps, the I impulses sit at the I ticks (n % sps == 0) and the Q
 * impulses at the Q ticks (n % sps == sps/2) — GLUE, parity unpinned by the reference. */
size_t or_tx_chain_src(or_phasor* p, const uint8_t* bits, size_t nbits, size_t sps,
                       const float* taps, size_t ntaps, float sample_freq, uint64_t s0,
                       size_t flush_syms, int out_mode, int even_odd, float* out);

/* RX chain, Demodulator loop structure: per input sample carrier.next() -> mix (complex
 * conjugate, or the reference's real-input mix with the 2x gain) -> FIRFilter on I and
 * Q at full rate -> keep n = k*sps + D -> slicer. Returns the number of symbols. */
size_t or_rx_chain(const float* x_iq, size_t n, float sample_freq, uint64_t s0, int mix,
                   const float* taps, size_t ntaps, size_t sps, size_t D,
                   const or_slicer* slicer, float* out_iq, uint8_t* out_sym, size_t cap);

/* modulate.rs:20-134 restated for one invocation: ASCII bits in, f32 samples out.
 * mod_name as in modulate.rs:74-95 (memoryless + dcqpsk/dqpsk/dbpsk kinds supported).
 * Returns the number of floats written, or -1 where the reference panics. */
long  or_modulate_cli(const char* mod_name, size_t sr, size_t br, size_t cf, size_t pc,
                      int iq, const char* text, size_t len, float* out, size_t cap);

#ifdef __cplusplus
}
#endif
#endif
