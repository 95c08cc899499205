// rust-modem_amd/cli/demodulate.cpp — the reference's `demodulate` binary (src/bin/demodulate.rs)
// on the MI355X backend, through the C ABI of include/modem_hip.h:
// native-endian i16 samples on stdin -> "i:{}\tq:{}" lines on stdout, byte for byte.
//
//   demodulate [-h] [-b RATE]
//
// demodulate.rs:15-44: the input is read two bytes at a time (bin/util.rs:3-37: reading stops
// at the first short read; for a file, an odd trailing byte); the analytic signal (x,
// hilbert(x)) feeds Demodulator::new(Carrier(900 Hz at 10 kHz), .., lowpass); lock_phase runs
// the PLL over the first 64 samples (demodulator.rs:32-36); every later sample gives one line
// (demodulator.rs:44-56, println! at demodulate.rs:41-43). Here: the Hilbert filter on
// modem_fir (bit-identical FIRFilter), the 64-sample PLL on modem_pll_lock (host, the
// reference's f32 operations), the demodulator on modem_rx with MODEM_MIX_REFERENCE_REAL_EXACT
// and MODEM_DTYPE_I16 (glibc-exact cos / sin, the FIRFilter fold), formatting as Rust's f32
// Display (fmt_f32.h). -b is accepted and unused, as in the reference. Panics of the reference
// (an unknown option, fewer than 64 samples for the lock) exit with status 101.
//
// Streaming, as the reference's iterator chain is: stdin is read as Rust's Stdin reads it (a
// BufReader of 8 KiB that refills with one read(2) only when empty, and a two-byte read that
// gets one byte ends the stream: bin/util.rs:13-24), the samples of each refill (several
// refills while more input is already waiting, up to kChunk samples) go through
// modem_rx_process, and their lines are written and flushed before the next read blocks — a
// live pipe sees its lines as its samples arrive, and memory stays bounded.
#include "../../include/modem_hip.h"
#include "demod_taps.h"
#include "fmt_f32.h"

#include <poll.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

const uint64_t kSampleRate = 10000;                          // demodulate.rs:10
const uint64_t kCarrier = 900;                               // demodulate.rs:36
const size_t kLock = 64;                                     // demodulator.rs:5
const size_t kChunk = (size_t)1 << 22;                       // samples per modem_rx_process call

[[noreturn]] void panic(const std::string& msg) {
    std::fflush(stdout);
    std::fprintf(stderr, "thread 'main' panicked at '%s'\n", msg.c_str());
    std::exit(101);
}

void check(modem_status s, const char* what) {
    if (s == MODEM_OK) return;
    std::fflush(stdout);
    std::fprintf(stderr, "demodulate: %s: %s\n", what, modem_status_str(s));
    std::exit(3);
}

// Rust's Stdin as bin/util.rs reads it: an 8 KiB BufReader (refilled by one read(2) when it is
// empty) and read_i16, whose two-byte read ends the stream when it gets fewer than two bytes.
struct StdinI16 {
    unsigned char buf[8192];
    size_t pos = 0, len = 0;
    bool done = false;
    // One refill's worth of samples appended to `out` (false: the stream has ended).
    bool refill(std::vector<int16_t>& out) {
        if (done) return false;
        ssize_t k;
        do k = ::read(0, buf, sizeof buf); while (k < 0 && errno == EINTR);
        if (k <= 0) { done = true; return false; }
        len = (size_t)k;
        pos = 0;
        const size_t ns = len / 2;
        const size_t at = out.size();
        out.resize(at + ns);
        if (ns) std::memcpy(out.data() + at, buf, ns * 2);   // std::mem::transmute: native endian
        pos = ns * 2;
        if (pos < len) done = true;                          // one byte left: Ok(1) -> end of input
        return ns > 0 || !done;
    }
    // More input can be read without blocking.
    static bool ready() {
        pollfd p{0, POLLIN, 0};
        return ::poll(&p, 1, 0) > 0 && (p.revents & (POLLIN | POLLHUP));
    }
};

void print_lines(const float* iq, size_t n, std::vector<char>& out) {
    char line[160];
    for (size_t k = 0; k < n; ++k) {
        int m = 0;
        std::memcpy(line, "i:", 2); m = 2;
        m += fmt_f32(line + m, iq[2 * k]);
        std::memcpy(line + m, "\tq:", 3); m += 3;
        m += fmt_f32(line + m, iq[2 * k + 1]);
        line[m++] = '\n';
        out.insert(out.end(), line, line + m);
        if (out.size() > ((size_t)1 << 20)) { std::fwrite(out.data(), 1, out.size(), stdout); out.clear(); }
    }
    std::fwrite(out.data(), 1, out.size(), stdout);
    out.clear();
    std::fflush(stdout);
}

}  // namespace

int main(int argc, char** argv) {
    for (int i = 1; i < argc; ++i) {                         // getopts: -h, -b RATE
        const char* a = argv[i];
        if (!std::strcmp(a, "-h") || !std::strcmp(a, "--help")) {
            std::printf("Usage: demodulate [-h] [-b RATE]\n\n    Demodulate a waveform on stdin to i/q samples on stdout\n\n"
                        "Options:\n    -h, --help          show usage\n    -b RATE             baud rate (symbols/sec)\n");
            return 0;
        }
        if (!std::strcmp(a, "-b")) {
            if (i + 1 >= argc) panic("called `Result::unwrap()` on an `Err` value: ArgumentMissing(\"b\")");
            ++i;
        } else if (std::strncmp(a, "-b", 2) != 0 && a[0] == '-' && a[1] != 0) {
            panic(std::string("called `Result::unwrap()` on an `Err` value: UnrecognizedOption(\"") + (a + 1) + "\")");
        }
    }
    StdinI16 in;
    std::vector<int16_t> x;
    while (x.size() < kLock && in.refill(x)) {}
    if (x.size() < kLock) panic("called `Option::unwrap()` on a `None` value");   // lock_phase
    const float w = modem_freq_sample_freq(kCarrier, kSampleRate);

    // lock_phase: the analytic signal of the first 64 samples through the PLL
    std::vector<float> xf(kLock), hil(kLock), xiq(2 * kLock);
    for (size_t k = 0; k < kLock; ++k) xf[k] = (float)x[k];
    modem_fir* hf;
    check(modem_fir_create(kDemodHilbert, 23, 0, &hf), "hilbert");
    check(modem_fir_process(hf, xf.data(), hil.data(), kLock, nullptr), "hilbert");
    check(modem_fir_destroy(hf), "hilbert");
    for (size_t k = 0; k < kLock; ++k) { xiq[2 * k] = xf[k]; xiq[2 * k + 1] = hil[k]; }
    float offset = 0.0f;
    check(modem_pll_lock(w, 0, xiq.data(), kLock, &offset), "pll");

    // the demodulator over the rest: carrier from sample 64, fresh low-pass filters
    modem_rx_desc d{};
    d.sample_freq = w;
    d.s0 = kLock;
    d.taps = kDemodLowpass;
    d.ntaps = 64;
    d.decim = 1;
    d.decim_offset = 0;
    d.mix = MODEM_MIX_REFERENCE_REAL_EXACT;
    d.in_dtype = MODEM_DTYPE_I16;
    d.out_dtype = MODEM_DTYPE_F32;
    d.slicer.kind = MODEM_SLICER_NONE;
    d.phase_offset = offset;
    modem_rx* rx;
    check(modem_rx_create(&d, 0, &rx), "rx");
    x.erase(x.begin(), x.begin() + kLock);
    std::vector<float> iq;
    std::vector<char> out;
    out.reserve((size_t)1 << 20);
    for (;;) {
        // what is already waiting joins this call (bounded), then the call's lines go out
        while (x.size() < kChunk && StdinI16::ready() && in.refill(x)) {}
        if (!x.empty()) {
            const size_t n = x.size();
            iq.resize(2 * n);
            size_t got = 0;
            check(modem_rx_process(rx, x.data(), n, iq.data(), nullptr, n, &got, nullptr), "rx");
            print_lines(iq.data(), got, out);
            x.clear();
        }
        if (!in.refill(x) && x.empty()) break;               // blocks until input or EOF
    }
    check(modem_rx_destroy(rx), "rx");
    return 0;
}
