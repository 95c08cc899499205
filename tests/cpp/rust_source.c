/* tests/cpp/rust_source.c — the Rust binding's Source-driven HipModulator (INTEGRATION.md,
 * `HipModulator::new(&mut carrier, phasor, Box<Source>, ...)`) restated in plain C, so that its
 * descriptor and its bit-gathering run against the real library where no `cargo` exists:
 *
 *  - `rust_tx_desc` declares the fields of the Rust `#[repr(C)] struct TxDesc` in the Rust
 *    order with the Rust field types; its layout is asserted equal to modem_tx_desc, and the
 *    handle is created from IT (q_offset = sps / 2 for EvenOddOffset, dtype, device);
 *  - the sources are data.rs's own state machines: Bits (data.rs:35-79), EvenOddOffset
 *    (data.rs:81-123) and AsciiBits (data.rs:125-186, whitespace skipped), each pulled once per
 *    sample as DigitalModulator::next does (modulator.rs:85-100);
 *  - HipModulator::pull: a Changed at a symbol tick appends the symbol's bits; a Changed at the
 *    half tick (EvenOddOffset) replaces the current symbol's bit 1; Finished ends the stream; the
 *    gathered bits go to modem_tx_process in chunks.
 *
 * Usage: rust_source <bits|evenodd|ascii> <out.f32> writes the `--iq` (i, q) stream (f32 LE) of
 * QPSK (bits, ascii) or OQPSK over EvenOddOffset (evenodd), sps 8, sample-and-hold, for a
 * built-in bit pattern; tests/test_gpu_parity.py::test_rust_source_binding compares it with
 * the oracle bit for bit. Exit 0 = ok.
 */
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "modem_hip.h"

/* ---- the Rust #[repr(C)] TxDesc, field for field ---- */
struct rust_tx_desc {
    uint32_t bits_per_symbol;   /* u32 */
    const float* lut;           /* *const f32 */
    uint32_t samples_per_symbol;
    const float* taps;
    uint32_t ntaps;
    float sample_freq;          /* f32 */
    uint64_t s0;                /* u64 */
    int32_t dtype;              /* i32 */
    int32_t out_mode;
    uint32_t q_offset;
    const void* phasor;         /* *const c_void */
};
#define SAME(f) _Static_assert(offsetof(struct rust_tx_desc, f) == offsetof(modem_tx_desc, f), #f)
SAME(bits_per_symbol); SAME(lut); SAME(samples_per_symbol); SAME(taps); SAME(ntaps); SAME(sample_freq);
SAME(s0); SAME(dtype); SAME(out_mode); SAME(q_offset); SAME(phasor);
_Static_assert(sizeof(struct rust_tx_desc) == sizeof(modem_tx_desc), "size");
_Static_assert(_Alignof(struct rust_tx_desc) == _Alignof(modem_tx_desc), "align");

/* ---- data.rs sources ---- */
enum { UNCHANGED, CHANGED, FINISHED };
typedef struct { size_t sps, counter; } symbol_clock;                  /* data.rs:14-33 */
static void clock_init(symbol_clock* c, size_t sps) { c->sps = sps; c->counter = sps - 1; }
static int clock_next(symbol_clock* c) { c->counter = (c->counter + 1) % c->sps; return c->counter == 0; }

typedef struct source source;
struct source { int (*next)(source*, const uint8_t**); };

typedef struct { source s; const uint8_t* bits; size_t n, bps, idx; symbol_clock clk; } bits_src;   /* :35-79 */
static int bits_next(source* s_, const uint8_t** out) {
    bits_src* s = (bits_src*)s_;
    if (clock_next(&s->clk)) {
        s->idx += 1;
        const size_t start = (s->idx - 1) * s->bps;
        if (start + s->bps > s->n) return FINISHED;
        *out = s->bits + start;
        return CHANGED;
    }
    *out = s->bits + (s->idx - 1) * s->bps;    /* bits().unwrap(): the current symbol */
    return UNCHANGED;
}

typedef struct { source s; source* data; symbol_clock clk; uint8_t cur[2]; } evenodd_src;     /* :81-123 */
static int evenodd_next(source* s_, const uint8_t** out) {
    evenodd_src* s = (evenodd_src*)s_;
    const uint8_t* b;
    const int u = s->data->next(s->data, &b);
    if (u == FINISHED) return FINISHED;
    if (u == CHANGED) {
        clock_next(&s->clk);
        s->cur[0] = b[0];
        *out = s->cur;
        return CHANGED;
    }
    *out = s->cur;
    if (clock_next(&s->clk)) { s->cur[1] = b[1]; return CHANGED; }
    return UNCHANGED;
}

typedef struct { source s; const char* text; size_t pos, len; symbol_clock clk; uint8_t bits[8]; size_t bps; } ascii_src;
static int ascii_bit(ascii_src* s, uint8_t* b) {                         /* :142-160 */
    while (s->pos < s->len) {
        const char c = s->text[s->pos++];
        if (c == ' ' || c == '\n' || c == '\t' || c == '\r') continue;
        if (c != '0' && c != '1') { fprintf(stderr, "assert!(is_digit(2)) failed\n"); exit(101); }
        *b = (uint8_t)(c - '0');
        return 1;
    }
    return 0;
}
static int ascii_next(source* s_, const uint8_t** out) {                 /* :174-186 */
    ascii_src* s = (ascii_src*)s_;
    *out = s->bits;
    if (clock_next(&s->clk)) {
        for (size_t i = 0; i < s->bps; ++i)
            if (!ascii_bit(s, &s->bits[i])) return FINISHED;
        return CHANGED;
    }
    return UNCHANGED;
}

/* ---- the binding: HipModulator::pull, restated ---- */
#define CHUNK_SYMBOLS 1000           /* small, so that the stream crosses several process calls */
typedef struct { modem_tx* h; size_t bps, sps, half; source* src; int finished; uint8_t* bits; size_t nbits; } hip_mod;

static void hm_pull(hip_mod* m) {
    m->nbits = 0;
    while (!m->finished && m->nbits < CHUNK_SYMBOLS * m->bps) {
        for (size_t j = 0; j < m->sps; ++j) {
            const uint8_t* b;
            const int u = m->src->next(m->src, &b);
            if (u == FINISHED) { m->finished = 1; break; }
            if (u == CHANGED) {
                if (j == 0) {                              /* a symbol tick: the symbol's bits */
                    memcpy(m->bits + m->nbits, b, m->bps);
                    m->nbits += m->bps;
                } else if (m->half && j == m->half) {     /* EvenOddOffset's half tick: bit 1 */
                    m->bits[m->nbits - m->bps + 1] = b[1];
                } else {
                    fprintf(stderr, "panic: Source changed off a symbol tick\n");
                    exit(101);
                }
            } else if (j == 0) {
                fprintf(stderr, "panic: no new symbol at a symbol tick\n");
                exit(101);
            }
        }
    }
}

#define CHECK(x) do { modem_status s_ = (x); if (s_ != MODEM_OK) { \
    fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, modem_status_str(s_)); return 1; } } while (0)

int main(int argc, char** argv) {
    if (argc != 3) { fprintf(stderr, "usage: rust_source <bits|evenodd|ascii> <out.f32>\n"); return 2; }
    enum { BPS = 2, SPS = 8, NSYM = 4099 };
    const int even_odd = strcmp(argv[1], "evenodd") == 0, ascii = strcmp(argv[1], "ascii") == 0;
    /* the bit pattern: xorshift bits, NSYM symbols plus one leftover bit (Bits stops at Finished) */
    const size_t nb = (size_t)NSYM * BPS + 1;
    uint8_t* raw = malloc(nb);
    uint64_t st = 0x2545F4914F6CDD1Dull;
    for (size_t i = 0; i < nb; ++i) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; raw[i] = (uint8_t)(st >> 63); }
    char* text = malloc(3 * nb + 1);
    size_t tl = 0;
    for (size_t i = 0; i < nb; ++i) { text[tl++] = (char)('0' + raw[i]); if (i % 7 == 6) text[tl++] = i % 21 == 20 ? '\n' : ' '; }

    /* OQPSK (modulate.rs "oqpsk": EvenOddOffset source) or QPSK; LUT from the phasor */
    const modem_phasor_desc ph = {.kind = even_odd ? MODEM_PHASOR_OQPSK : MODEM_PHASOR_QPSK, .bits_per_symbol = BPS,
                                  .phase = 0.f, .amplitude = 1.f};
    float lut[2 << BPS];
    CHECK(modem_phasor_lut(&ph, lut));
    const struct rust_tx_desc d = {.bits_per_symbol = BPS, .lut = lut, .samples_per_symbol = SPS, .taps = NULL, .ntaps = 0,
                                   .sample_freq = modem_freq_sample_freq(1000, 10000), .s0 = 0, .dtype = 0,
                                   .out_mode = MODEM_OUT_IQ_BASEBAND, .q_offset = even_odd ? SPS / 2 : 0, .phasor = NULL};
    modem_tx* h;
    CHECK(modem_tx_create((const modem_tx_desc*)&d, /*device*/ 0, &h));

    bits_src bs = {{bits_next}, raw, nb, BPS, 0, {0, 0}};
    clock_init(&bs.clk, SPS);
    evenodd_src eo = {{evenodd_next}, &bs.s, {0, 0}, {0, 0}};
    clock_init(&eo.clk, SPS / BPS);
    ascii_src as = {{ascii_next}, text, 0, tl, {0, 0}, {0}, BPS};
    clock_init(&as.clk, SPS);
    hip_mod m = {h, BPS, SPS, even_odd ? SPS / 2 : 0, even_odd ? &eo.s : ascii ? &as.s : &bs.s, 0,
                 malloc((CHUNK_SYMBOLS + 1) * BPS), 0};
    float* y = malloc(2 * sizeof(float) * (size_t)(NSYM + 1) * SPS);
    size_t n = 0, calls = 0;
    for (;;) {
        hm_pull(&m);
        if (m.nbits == 0) break;
        size_t got;
        CHECK(modem_tx_process(h, m.bits, m.nbits, y + 2 * n, m.nbits / BPS * SPS, &got, NULL));
        n += got;
        ++calls;
    }
    if (modem_tx_sample(h) != n) { fprintf(stderr, "carrier sample %llu != %zu\n", (unsigned long long)modem_tx_sample(h), n); return 1; }
    CHECK(modem_tx_destroy(h));
    FILE* f = fopen(argv[2], "wb");
    if (!f || fwrite(y, sizeof(float), 2 * n, f) != 2 * n) return 1;
    fclose(f);
    char bp[4096];
    snprintf(bp, sizeof bp, "%s.bits", argv[2]);           /* the bit pattern, for the oracle */
    f = fopen(bp, "wb");
    if (!f || fwrite(raw, 1, nb, f) != nb) return 1;
    fclose(f);
    printf("rust_source %s: %zu samples in %zu process calls\n", argv[1], n, calls);
    free(raw); free(text); free(m.bits); free(y);
    return n == (size_t)NSYM * SPS ? 0 : 1;
}
