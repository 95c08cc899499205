/* tests/cpp/loopback.c — the C ABI driven from plain C, as a non-Python host would (no HIP
 * headers, host buffers): 16-QAM, sps 4, 129-tap RRC TX -> RX over 2^16 symbols, in two
 * process calls per side plus the flushes. Checks that every decision equals the symbol sent
 * and that the handles report the sample counters the reference's Carrier would hold.
 * Exit 0 = pass. Run by tests/test_gpu_parity.py::test_c_host_loopback (needs the GPU).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "modem_hip.h"

#define CHECK(x) do { modem_status s_ = (x); if (s_ != MODEM_OK) { \
    fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, modem_status_str(s_)); return 1; } } while (0)

int main(void) {
    enum { BPS = 4, SPS = 4, L = 129, NSYM = 1 << 16 };
    if (modem_abi_version() != MODEM_HIP_ABI_VERSION) {
        fprintf(stderr, "library ABI %d, header %d\n", (int)modem_abi_version(), MODEM_HIP_ABI_VERSION);
        return 1;
    }
    const modem_phasor_desc qam = {.kind = MODEM_PHASOR_QAM, .bits_per_symbol = BPS, .phase = 0.f, .amplitude = 1.f};
    float lut[2 << BPS], taps[L];
    CHECK(modem_phasor_lut(&qam, lut));
    CHECK(modem_rrc_taps(L, SPS, 0.35, taps));
    const float w = modem_freq_sample_freq(1, 4);

    uint8_t* bits = malloc((size_t)NSYM * BPS);
    uint8_t* sent = malloc(NSYM);
    uint64_t st = 0x9E3779B97F4A7C15ull;
    for (size_t k = 0; k < NSYM; ++k) {
        st ^= st << 13; st ^= st >> 7; st ^= st << 17;
        sent[k] = (uint8_t)(st >> 60);
        for (int b = 0; b < BPS; ++b) bits[k * BPS + b] = (sent[k] >> (BPS - 1 - b)) & 1;   /* MSB first */
    }

    modem_tx_desc td = {.bits_per_symbol = BPS, .lut = lut, .samples_per_symbol = SPS, .taps = taps, .ntaps = L,
                        .sample_freq = w, .s0 = 0, .dtype = MODEM_DTYPE_F32, .out_mode = MODEM_OUT_IQ_MIXED};
    modem_tx* tx;
    CHECK(modem_tx_create(&td, 0, &tx));
    const size_t cap = (size_t)NSYM * SPS + 2 * L;
    float* y = malloc(2 * cap * sizeof(float));
    size_t n = 0, got;
    const size_t half = (size_t)NSYM / 2 * BPS + 3;          /* a split inside a symbol */
    CHECK(modem_tx_process(tx, bits, half, y, cap, &got, NULL));
    n += got;
    CHECK(modem_tx_process(tx, bits + half, (size_t)NSYM * BPS - half, y + 2 * n, cap - n, &got, NULL));
    n += got;
    CHECK(modem_tx_flush(tx, y + 2 * n, cap - n, &got, NULL));
    n += got;
    if (modem_tx_sample(tx) != n) { fprintf(stderr, "tx sample %llu != %zu\n", (unsigned long long)modem_tx_sample(tx), n); return 1; }

    modem_rx_desc rd = {.sample_freq = w, .s0 = 0, .taps = taps, .ntaps = L, .decim = SPS, .decim_offset = L - 1,
                        .mix = MODEM_MIX_COMPLEX, .in_dtype = MODEM_DTYPE_F32, .out_dtype = MODEM_DTYPE_F32};
    CHECK(modem_phasor_slicer(&qam, lut, &rd.slicer));
    modem_rx* rx;
    CHECK(modem_rx_create(&rd, 0, &rx));
    float* iq = malloc(2 * (size_t)NSYM * 2 * sizeof(float));
    uint8_t* sym = malloc((size_t)NSYM * 2);
    size_t k = 0;
    const size_t cut = 100003;                                /* not a multiple of anything */
    CHECK(modem_rx_process(rx, y, cut, iq, sym, (size_t)NSYM * 2, &got, NULL));
    k += got;
    CHECK(modem_rx_process(rx, y + 2 * cut, n - cut, iq + 2 * k, sym + k, (size_t)NSYM * 2 - k, &got, NULL));
    k += got;
    if (modem_rx_sample(rx) != n) { fprintf(stderr, "rx sample %llu != %zu\n", (unsigned long long)modem_rx_sample(rx), n); return 1; }
    if (k < NSYM) { fprintf(stderr, "only %zu decisions\n", k); return 1; }
    size_t bad = 0;
    for (size_t i = 0; i < NSYM; ++i) bad += sym[i] != sent[i];
    double emax = 0.0;                                        /* the constellation point it decided */
    for (size_t i = 0; i < NSYM; ++i) {
        const double dr = iq[2 * i] - lut[2 * sent[i]], di = iq[2 * i + 1] - lut[2 * sent[i] + 1];
        emax = fmax(emax, sqrt(dr * dr + di * di));
    }
    CHECK(modem_rx_destroy(rx));
    CHECK(modem_tx_destroy(tx));
    printf("loopback: %zu samples, %zu decisions, %zu wrong, max |r - lut[sent]| %.3g\n", n, k, bad, emax);
    free(bits); free(sent); free(y); free(iq); free(sym);
    return bad == 0 && emax < 0.05 ? 0 : 1;
}
