// rust-modem_amd/cli/modulate.cpp — the reference's `modulate` binary (src/bin/modulate.rs)
// on the MI355X backend: ASCII bits on stdin -> f32 little-endian samples on stdout, through
// the C ABI of include/modem_hip.h.
//
//   modulate -m MOD [-r RATE] [-b RATE] [-c FREQ] [-p CYCLES] [--iq]
//
// Same options, defaults and output as modulate.rs:20-134: --iq writes the (i, q) pairs of
// DigitalModulator (bit-identical, modulate.rs:109-116); otherwise an optional preamble of
// sr/cf*pc - 1 samples of the Raw phasor (modulate.rs:118-126) then the real part of the
// modulated data (modulate.rs:128-133), both on one carrier. Panics of the reference (missing
// or unparsable options, the asserts at modulate.rs:62,68, a non-binary digit on stdin at
// data.rs:155, an unknown modulation) exit with status 101, as a Rust panic does. Every
// modulation of modulate.rs:74-95 is supported.
#include "../../include/modem_hip.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

const float kAmplitude = 1.0f;                              // modulate.rs:14
const float kPi = 3.14159265358979323846f;                  // std::f32::consts::PI

[[noreturn]] void panic(const std::string& msg) {
    std::fflush(stdout);
    std::fprintf(stderr, "thread 'main' panicked at '%s'\n", msg.c_str());
    std::exit(101);
}

void check(modem_status s, const char* what) {
    if (s == MODEM_OK) return;
    if (s == MODEM_ERR_INVALID_ARG) panic(std::string(what) + ": " + modem_status_str(s));
    std::fflush(stdout);
    std::fprintf(stderr, "modulate: %s: %s\n", what, modem_status_str(s));
    std::exit(3);
}

size_t parse_usize(const std::string& v, const char* what) {
    // Rust's usize::parse: optional '+', decimal digits only, no overflow
    size_t i = (!v.empty() && v[0] == '+') ? 1 : 0;
    if (i == v.size()) panic(what);
    unsigned long long x = 0;
    for (; i < v.size(); ++i) {
        if (v[i] < '0' || v[i] > '9') panic(what);
        const unsigned long long d = (unsigned long long)(v[i] - '0');
        if (x > (~0ull - d) / 10) panic(what);
        x = x * 10 + d;
    }
    return (size_t)x;
}

// `(byte as char).is_whitespace()` for a byte: ASCII whitespace plus U+0085 and U+00A0.
bool is_ws(unsigned char c) {
    return c == ' ' || (c >= 0x09 && c <= 0x0d) || c == 0x85 || c == 0xa0;
}

struct Opts {
    std::string mod;
    bool have_mod = false, iq = false, help = false;
    std::string r, b, c, p;
    bool have_r = false, have_b = false, have_c = false, have_p = false;
};

Opts parse_args(int argc, char** argv) {
    Opts o;
    auto take = [&](int& i, const char* flag, std::string& dst, bool& have) {
        const size_t fl = std::strlen(flag);
        const char* a = argv[i];
        if (std::strlen(a) > fl) { dst = a + fl; have = true; return; }   // -mqpsk
        if (i + 1 >= argc) panic(std::string("Argument to option '") + (flag + 1) + "' missing.");
        dst = argv[++i];
        have = true;
    };
    for (int i = 1; i < argc; ++i) {
        const char* a = argv[i];
        if (!std::strcmp(a, "-h") || !std::strcmp(a, "--help")) o.help = true;
        else if (!std::strcmp(a, "--iq")) o.iq = true;
        else if (!std::strncmp(a, "-m", 2)) take(i, "-m", o.mod, o.have_mod);
        else if (!std::strncmp(a, "-r", 2)) take(i, "-r", o.r, o.have_r);
        else if (!std::strncmp(a, "-b", 2)) take(i, "-b", o.b, o.have_b);
        else if (!std::strncmp(a, "-c", 2)) take(i, "-c", o.c, o.have_c);
        else if (!std::strncmp(a, "-p", 2)) take(i, "-p", o.p, o.have_p);
        else panic(std::string("Unrecognized option: '") + a + "'.");
    }
    return o;
}

// The phasors of modulate.rs:74-95 as descriptors: memoryless ones become a LUT
// (modem_phasor_lut), sample-dependent ones (dcqpsk, msk, 16cpfsk) go to the TX handle as
// modem_tx_desc.phasor. `offset`: the EvenOddOffset source (modulate.rs:101-107).
bool phasor_for(const std::string& m, size_t sr, size_t br, size_t sps, modem_phasor_desc& d,
                std::vector<modem_ring>& rings, bool& offset) {
    std::memset(&d, 0, sizeof d);
    d.amplitude = kAmplitude;
    offset = false;
    if (m == "dcqpsk") { d.kind = MODEM_PHASOR_DCQPSK; return true; }                  // :86
    if (m == "msk") {                                                                   // :81
        if (sps % 2 != 0) panic("assertion failed: samples_per_symbol % 2 == 0");       // msk.rs:14
        d.kind = MODEM_PHASOR_MSK; d.samples_per_symbol = (uint32_t)sps; offset = true;
        return true;
    }
    if (m == "16cpfsk") {                                                               // :87
        d.kind = MODEM_PHASOR_CPFSK; d.bits_per_symbol = 4;
        d.freq = modem_freq_sample_freq(1 * br / 2, sr);                                // cpfsk.rs:20-21
        return true;
    }
    if (m == "bfsk") { d.kind = MODEM_PHASOR_BFSK; d.freq = modem_freq_sample_freq(200, sr); return true; } // :77
    if (m == "mfsk") {                                                                  // :82-83
        d.kind = MODEM_PHASOR_MFSK; d.bits_per_symbol = 4; d.freq = modem_freq_sample_freq(50, sr);
        d.mfsk_map = 1;                                                                 // IncreaseMap
        return true;
    }
    if (m == "dqpsk" || m == "dbpsk") {                                                 // :92-93
        d.kind = MODEM_PHASOR_DMPSK; d.bits_per_symbol = m == "dqpsk" ? 2 : 1;
        d.phase = kPi / 4.0f; d.shift = m == "dqpsk" ? kPi / 2.0f : kPi;
        return true;
    }
    if (m == "bask") { d.kind = MODEM_PHASOR_BASK; return true; }
    if (m == "bpsk") { d.kind = MODEM_PHASOR_BPSK; d.phase = kPi / 4.0f; return true; }
    if (m == "qpsk") { d.kind = MODEM_PHASOR_QPSK; d.phase = 0.0f; return true; }
    if (m == "qam16") { d.kind = MODEM_PHASOR_QAM; d.bits_per_symbol = 4; return true; }
    if (m == "qam256") { d.kind = MODEM_PHASOR_QAM; d.bits_per_symbol = 8; return true; }
    if (m == "16psk") { d.kind = MODEM_PHASOR_MPSK; d.bits_per_symbol = 4; d.phase = 0.0f; return true; }
    if (m == "oqpsk") { d.kind = MODEM_PHASOR_OQPSK; offset = true; return true; }   // modulate.rs:101-107
    if (m == "16apsk") {                                                                  // modulate.rs:88-91
        rings = {{0, 4, 0.5f, kPi / 4.0f}, {4, 16, 1.0f, kPi / 12.0f}};
        d.kind = MODEM_PHASOR_APSK;
        d.bits_per_symbol = 4;
        d.nrings = 2;
        d.rings = rings.data();
        return true;
    }
    return false;
}

void write_floats(const std::vector<float>& v, size_t n) {
    // f32 little-endian (byteorder::LittleEndian; the host is little-endian)
    if (n && std::fwrite(v.data(), sizeof(float), n, stdout) != n) std::exit(1);
}

}  // namespace

int main(int argc, char** argv) {
    const Opts o = parse_args(argc, argv);
    if (o.help) {
        std::printf("Usage: modulate [-h] [-m MOD] [-r RATE] [-b RATE] [-c FREQ] [-p CYCLES] [--iq]\n\n"
                    "    Modulate the bits on stdin to a waveform on stdout\n");
        return 0;
    }
    if (!o.have_mod) panic("digital modulation is required");
    const size_t sr = o.have_r ? parse_usize(o.r, "invalid sample rate") : 10000;
    const size_t br = o.have_b ? parse_usize(o.b, "invalid baud rate") : 220;
    const size_t cf = o.have_c ? parse_usize(o.c, "invalid carrier frequency") : 1000;
    size_t pc = 0;
    if (o.have_p) {
        if (cf == 0) panic("attempt to calculate the remainder with a divisor of zero");
        if (sr % cf != 0) panic("assertion failed: sr % cf == 0");                     // modulate.rs:62
        pc = parse_usize(o.p, "invalid preamble cycles");
    }
    if (!(cf < sr / 2)) panic("assertion failed: cf < sr / 2");                         // modulate.rs:68
    uint64_t sps = 0;
    if (modem_rates_sps(br, sr, &sps) != MODEM_OK) panic("attempt to divide by zero");  // rates.rs:12-18
    const float w = modem_freq_sample_freq(cf, sr);                                     // modulate.rs:71

    modem_phasor_desc pd;
    std::vector<modem_ring> rings;
    bool offset = false;
    if (!phasor_for(o.mod, sr, br, sps, pd, rings, offset))
        panic("invalid digital modulation");                                            // modulate.rs:94
    uint32_t bps = 0;
    check(modem_phasor_bits(&pd, &bps), "phasor");
    const bool per_sample = pd.kind == MODEM_PHASOR_DCQPSK || pd.kind == MODEM_PHASOR_MSK ||
                            pd.kind == MODEM_PHASOR_CPFSK || pd.kind == MODEM_PHASOR_DMPSK ||
                            pd.kind == MODEM_PHASOR_MFSK || pd.kind == MODEM_PHASOR_BFSK;
    std::vector<float> lut(2u << bps);
    if (!per_sample) check(modem_phasor_lut(&pd, lut.data()), "phasor");
    if (offset && sps % 2 != 0) panic("assertion failed: samples_per_symbol % bits_per_symbol == 0");

    uint64_t s0 = 0;                                   // the carrier shared by preamble and data
    if (!o.iq && pc > 0) {                             // modulate.rs:118-126: Raw phasor (A, 0)
        const size_t nt = sr / cf * pc - 1;
        const float raw[4] = {kAmplitude, 0.0f, kAmplitude, 0.0f};
        modem_tx_desc d{};
        d.bits_per_symbol = 1;
        d.lut = raw;
        d.samples_per_symbol = 1;
        d.sample_freq = w;
        d.dtype = MODEM_DTYPE_F32;
        d.out_mode = MODEM_OUT_REAL;
        modem_tx* h = nullptr;
        check(modem_tx_create(&d, 0, &h), "preamble");
        std::vector<uint8_t> zeros(1 << 20, 0);
        std::vector<float> out(zeros.size());
        for (size_t done = 0; done < nt;) {
            const size_t n = nt - done < zeros.size() ? nt - done : zeros.size();
            size_t got = 0;
            check(modem_tx_process(h, zeros.data(), n, out.data(), out.size(), &got, nullptr), "preamble");
            write_floats(out, got);
            done += n;
        }
        s0 = modem_tx_sample(h);
        modem_tx_destroy(h);
    }

    modem_tx_desc d{};
    d.bits_per_symbol = bps;
    d.lut = lut.data();
    d.samples_per_symbol = (uint32_t)sps;
    d.ntaps = 0;                                       // DigitalModulator: sample-and-hold
    d.sample_freq = w;
    d.s0 = s0;
    d.dtype = MODEM_DTYPE_F32;
    d.out_mode = o.iq ? MODEM_OUT_IQ_BASEBAND : MODEM_OUT_REAL;
    d.q_offset = offset ? (uint32_t)(sps / 2) : 0;
    d.phasor = per_sample ? &pd : nullptr;
    modem_tx* h = nullptr;
    check(modem_tx_create(&d, 0, &h), "modulator");

    // AsciiBits (data.rs:125-185): whitespace is skipped, anything else must be '0' or '1'.
    // Bits go to the device in chunks; a bad digit ends the stream after the symbols that
    // precede it, then panics (data.rs:155).
    const size_t kChunk = (size_t)1 << 22;
    std::vector<uint8_t> bits;
    bits.reserve(kChunk);
    std::vector<float> out;
    bool bad = false;
    auto flush_bits = [&](bool last) {
        if (bits.empty()) return;
        // keep whole symbols together with a panic at the exact point the reference stops
        const size_t per = o.iq ? 2 : 1;
        const size_t cap = (bits.size() / bps + 1) * sps;
        if (out.size() < cap * per) out.resize(cap * per);
        size_t got = 0;
        check(modem_tx_process(h, bits.data(), bits.size(), out.data(), cap, &got, nullptr), "modulator");
        write_floats(out, got * per);
        bits.clear();
        (void)last;
    };
    unsigned char buf[1 << 16];
    for (;;) {
        const size_t n = std::fread(buf, 1, sizeof buf, stdin);
        if (n == 0) break;
        for (size_t i = 0; i < n; ++i) {
            const unsigned char ch = buf[i];
            if (is_ws(ch)) continue;
            if (ch != '0' && ch != '1') { bad = true; break; }
            bits.push_back((uint8_t)(ch - '0'));
            if (bits.size() >= kChunk) flush_bits(false);
        }
        if (bad) break;
    }
    flush_bits(true);                                  // leftover bits (< bps) never form a symbol
    modem_tx_destroy(h);
    std::fflush(stdout);
    if (bad) panic("assertion failed: (bit as char).is_digit(2)");
    return 0;
}
