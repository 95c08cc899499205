// rust-modem_amd/csrc/modem_capi.cpp — implementation of include/modem_hip.h.
//
// Host side of the drop-in boundary: phasor LUT builders (the memoryless DigitalPhasor
// plugins evaluated once per symbol value, same expressions and rounding as the reference),
// RRC tap generation, and the streaming TX / RX / FIR handles that own device state and
// launch the kernels of modem_kernels.hip. Built with -ffp-contract=off so host float
// expressions round like rustc's.
#include "../../include/modem_hip.h"
#include "modem_internal.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#pragma clang fp contract(off)

namespace {

constexpr float kPi = 3.14159265358979323846f;   // std::f32::consts::PI

struct DeviceGuard {   // scoped hipSetDevice (no call when the device is already current)
    int old = -1;
    bool ok = false, set = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&old) != hipSuccess) { (void)hipGetLastError(); old = -1; }
        if (old == dev) { ok = true; return; }
        ok = hipSetDevice(dev) == hipSuccess;
        set = ok;
        if (!ok) (void)hipGetLastError();
    }
    ~DeviceGuard() { if (set && old >= 0) (void)hipSetDevice(old); }
};

bool is_device_ptr(const void* p) {
    if (!p) return false;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) { (void)hipGetLastError(); return false; }
    return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

// Device memory of a GPU other than `dev` (managed memory is reachable from every device).
// A handle's kernels run on its own device: such a buffer would be read over the fabric or
// fault, so the entry points refuse it (the reference has one address space, no counterpart).
bool foreign_ptr(const void* p, int dev) {
    if (!p) return false;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) { (void)hipGetLastError(); return false; }
    return a.type == hipMemoryTypeDevice && a.device != dev;
}

// Both facts from one attribute query (the per-call host cost of a process() is mostly these
// queries): host memory (staged), device memory the handle's kernels can use, or another
// GPU's memory (refused).
enum PtrKind { PTR_HOST = 0, PTR_DEVICE = 1, PTR_FOREIGN = 2 };
PtrKind ptr_kind(const void* p, int dev) {
    if (!p) return PTR_HOST;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) { (void)hipGetLastError(); return PTR_HOST; }
    if (a.type == hipMemoryTypeManaged) return PTR_DEVICE;
    if (a.type != hipMemoryTypeDevice) return PTR_HOST;
    return a.device == dev ? PTR_DEVICE : PTR_FOREIGN;
}

#define HIP_TRY(expr)                                                              \
    do {                                                                           \
        if ((expr) != hipSuccess) { (void)hipGetLastError(); return MODEM_ERR_HIP; } \
    } while (0)

template <typename T>
modem_status dalloc(T** p, size_t count) {
    *p = nullptr;
    if (count == 0) count = 1;
    if (hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T)) != hipSuccess) {
        (void)hipGetLastError();
        *p = nullptr;
        return MODEM_ERR_ALLOC;
    }
    if (hipMemset(*p, 0, count * sizeof(T)) != hipSuccess) { (void)hipGetLastError(); return MODEM_ERR_HIP; }
    return MODEM_OK;
}

// Growable device staging buffer for host-pointer I/O.
struct Stage {
    void* p = nullptr;
    size_t cap = 0;
    modem_status ensure(size_t bytes) {
        if (bytes <= cap) return MODEM_OK;
        if (p) (void)hipFree(p);
        p = nullptr; cap = 0;
        if (hipMalloc(&p, bytes) != hipSuccess) { (void)hipGetLastError(); p = nullptr; return MODEM_ERR_ALLOC; }
        cap = bytes;
        return MODEM_OK;
    }
    ~Stage() { if (p) (void)hipFree(p); }
};

bool device_ok(int device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) { (void)hipGetLastError(); return false; }
    return device >= 0 && device < n;
}

// ---- reference restatements used by the LUT builder (digital/util.rs, util.rs) ----------
float bit_to_sign(uint8_t b) { return (float)(int8_t)(2 * (int8_t)b - 1); }   // digital/util.rs:1-3
uint8_t bytes_to_bits(const uint8_t* b, size_t n) {                            // digital/util.rs:5-11
    if (n == 0) return 0;
    uint8_t s = 0;
    for (size_t i = 0; i < n; ++i) s = (uint8_t)(s | (uint8_t)((b[i] & 1) << (n - 1 - i)));
    return s;
}
float mod_trig(float x) {                                                      // util.rs:3-6
    const float two_pi = kPi * 2.0f;
    return x - two_pi * std::floor(x / two_pi);
}

modem_status phasor_bps(const modem_phasor_desc* d, uint32_t* bps) {
    switch (d->kind) {
    case MODEM_PHASOR_BPSK: case MODEM_PHASOR_BASK: *bps = 1; return MODEM_OK;
    case MODEM_PHASOR_QPSK: case MODEM_PHASOR_OQPSK: *bps = 2; return MODEM_OK;
    case MODEM_PHASOR_QAM:
        if (d->bits_per_symbol < 2 || d->bits_per_symbol > 8) return MODEM_ERR_INVALID_ARG;  // qam.rs:17
        *bps = d->bits_per_symbol; return MODEM_OK;
    case MODEM_PHASOR_MPSK: case MODEM_PHASOR_APSK: case MODEM_PHASOR_CPFSK: case MODEM_PHASOR_DMPSK:
    case MODEM_PHASOR_MFSK:
        if (d->bits_per_symbol < 1 || d->bits_per_symbol > 8) return MODEM_ERR_INVALID_ARG;
        *bps = d->bits_per_symbol; return MODEM_OK;
    case MODEM_PHASOR_DCQPSK: case MODEM_PHASOR_MSK: *bps = 2; return MODEM_OK;   // dcqpsk.rs:39, msk.rs:28
    case MODEM_PHASOR_BFSK: *bps = 1; return MODEM_OK;                            // bfsk.rs:23
    default: return MODEM_ERR_INVALID_ARG;
    }
}

bool phasor_scanned(int kind) {          // phase carried from symbol to symbol (tx_scan)
    return kind == MODEM_PHASOR_DMPSK || kind == MODEM_PHASOR_MFSK || kind == MODEM_PHASOR_BFSK;
}
bool phasor_sample_dependent(int kind) {
    return kind == MODEM_PHASOR_DCQPSK || kind == MODEM_PHASOR_CPFSK || kind == MODEM_PHASOR_MSK ||
           phasor_scanned(kind);
}

// i(_, b), q(_, b) of one memoryless phasor for the bit slice b (MSB first).
modem_status phasor_iq(const modem_phasor_desc* d, const uint8_t* b, size_t n, float* i, float* q) {
    const float A = d->amplitude;
    switch (d->kind) {
    case MODEM_PHASOR_BPSK: {                                     // bpsk.rs:17-31
        const float c = bit_to_sign(b[0]) * A;
        *i = c * std::cos(d->phase); *q = c * std::sin(d->phase);
        return MODEM_OK;
    }
    case MODEM_PHASOR_QPSK: {                                     // qpsk.rs:11-35
        const float pc = std::cos(d->phase), ps = std::sin(d->phase);
        const float amp = A * std::sqrt(0.5f);
        *i = amp * (bit_to_sign(b[0]) * pc - bit_to_sign(b[1]) * ps);
        *q = amp * (bit_to_sign(b[1]) * pc + bit_to_sign(b[0]) * ps);
        return MODEM_OK;
    }
    case MODEM_PHASOR_QAM: {                                      // qam.rs:15-60
        const size_t cs = n / 2;
        const float ms = (float)((1u << cs) - 1);
        const float pc = std::cos(d->phase), ps = std::sin(d->phase);
        const float amp = A / ms / 2.0f;
        const float pm = 2.0f * (float)bytes_to_bits(b, cs) - ms;
        const float pl = 2.0f * (float)bytes_to_bits(b + cs, n - cs) - ms;
        *i = amp * (pm * pc - pl * ps);
        *q = amp * (pl * pc + pm * ps);
        return MODEM_OK;
    }
    case MODEM_PHASOR_BASK:                                       // bask.rs:15-24
        *i = (float)b[0] * A; *q = 0.0f;
        return MODEM_OK;
    case MODEM_PHASOR_MPSK: {                                     // mpsk.rs:14-41
        const float ns = (float)(1u << n);
        const float inner = 2.0f * kPi * (float)bytes_to_bits(b, n) / ns + d->phase;
        *i = A * std::cos(inner); *q = A * std::sin(inner);
        return MODEM_OK;
    }
    case MODEM_PHASOR_APSK: {                                     // apsk.rs:36-56
        const uint8_t s = bytes_to_bits(b, n);
        const modem_ring* ring = nullptr;
        for (uint32_t k = 0; k < d->nrings; ++k)
            if (s >= d->rings[k].start && s < d->rings[k].end) { ring = &d->rings[k]; break; }
        if (!ring) return MODEM_ERR_INVALID_ARG;
        const float inner = 2.0f * kPi * (float)(uint8_t)(s - ring->start) /
                            (float)(uint8_t)(ring->end - ring->start) + ring->phase;
        *i = A * ring->radius * std::cos(inner); *q = A * ring->radius * std::sin(inner);
        return MODEM_OK;
    }
    case MODEM_PHASOR_OQPSK: {                                    // oqpsk.rs:9-25
        const float amp = A * std::sqrt(0.5f);
        *i = bit_to_sign(b[0]) * amp; *q = bit_to_sign(b[1]) * amp;
        return MODEM_OK;
    }
    default: return MODEM_ERR_INVALID_ARG;
    }
}

modem_status apsk_verify(const modem_phasor_desc* d, uint32_t bps) {   // apsk.rs:25-26,74,85-97
    if (d->nrings == 0 || !d->rings) return MODEM_ERR_INVALID_ARG;
    unsigned prev = 0;
    for (uint32_t k = 0; k < d->nrings; ++k) {
        const modem_ring& r = d->rings[k];
        if (!(r.radius >= 0.0f && r.radius <= 1.0f)) return MODEM_ERR_INVALID_ARG;
        if (r.start != prev) return MODEM_ERR_INVALID_ARG;
        prev = r.end;
    }
    return prev == (1u << bps) ? MODEM_OK : MODEM_ERR_INVALID_ARG;
}

}  // namespace

// =====================================================================================
extern "C" {

const char* modem_status_str(modem_status s) {
    switch (s) {
    case MODEM_OK: return "ok";
    case MODEM_ERR_INVALID_ARG: return "invalid argument (the reference would panic)";
    case MODEM_ERR_UNSUPPORTED: return "unsupported by this backend";
    case MODEM_ERR_HIP: return "HIP runtime error";
    case MODEM_ERR_NO_DEVICE: return "no such HIP device";
    case MODEM_ERR_CAPACITY: return "output buffer too small";
    case MODEM_ERR_ALLOC: return "allocation failed";
    }
    return "unknown status";
}

int32_t modem_abi_version(void) { return MODEM_HIP_ABI_VERSION; }

float modem_freq_sample_freq(uint64_t hz, uint64_t sr) {           // freq.rs:19-26
    const float ang = 2.0f * kPi * (float)hz;
    return ang / (float)sr;
}

modem_status modem_pll_lock(float w, uint64_t s0, const float* x, size_t n, float* off) {
    if (!off || (n && !x)) return MODEM_ERR_INVALID_ARG;
    const float change = 0.447214f;                                          // pll.rs:3
    for (size_t k = 0; k < n; ++k) {                                         // demodulator.rs:33-35
        const float inner = mod_trig(w * (float)(s0 + k)) + *off;            // pll.rs:17
        const float cr = std::cos(inner), ci = -std::sin(inner);             // Complex::new(cos, sin).conj()
        const float re = x[2 * k] * cr - x[2 * k + 1] * ci;                  // num::Complex Mul
        const float im = x[2 * k] * ci + x[2 * k + 1] * cr;
        *off += change * std::atan2(im, re);                                 // pll.rs:19-21
    }
    return MODEM_OK;
}

modem_status modem_rates_sps(uint64_t br, uint64_t sr, uint64_t* sps) {   // rates.rs:12-18
    if (!sps || br == 0) return MODEM_ERR_INVALID_ARG;
    *sps = sr / br;
    return MODEM_OK;
}

float modem_carrier_phase(float w, uint64_t n) { return mod_trig(w * (float)n); }   // carrier.rs:17-19

modem_status modem_carrier_phases(float w, uint64_t s0, size_t n, float* out, int device, void* stream) {
    if (n && (!out || !is_device_ptr(out) || foreign_ptr(out, device))) return MODEM_ERR_INVALID_ARG;
    if (!device_ok(device)) return MODEM_ERR_NO_DEVICE;
    DeviceGuard g(device);
    if (!g.ok) return MODEM_ERR_NO_DEVICE;
    HIP_TRY(mk::launch_phases(w, s0, n, out, (hipStream_t)stream));
    return MODEM_OK;
}

modem_status modem_phasor_bits(const modem_phasor_desc* d, uint32_t* bps) {
    if (!d || !bps) return MODEM_ERR_INVALID_ARG;
    return phasor_bps(d, bps);
}

modem_status modem_phasor_lut(const modem_phasor_desc* d, float* lut) {
    if (!d || !lut) return MODEM_ERR_INVALID_ARG;
    uint32_t bps;
    modem_status st = phasor_bps(d, &bps);
    if (st) return st;
    if (phasor_sample_dependent(d->kind)) return MODEM_ERR_UNSUPPORTED;   // no bits-only table
    if (d->kind == MODEM_PHASOR_APSK && (st = apsk_verify(d, bps))) return st;
    uint8_t b[8];
    for (uint32_t s = 0; s < (1u << bps); ++s) {
        for (uint32_t k = 0; k < bps; ++k) b[k] = (uint8_t)((s >> (bps - 1 - k)) & 1u);
        if ((st = phasor_iq(d, b, bps, &lut[2 * s], &lut[2 * s + 1]))) return st;
    }
    return MODEM_OK;
}

modem_status modem_phasor_slicer(const modem_phasor_desc* d, const float* lut, modem_slicer_desc* o) {
    if (!d || !o) return MODEM_ERR_INVALID_ARG;
    uint32_t bps;
    modem_status st = phasor_bps(d, &bps);
    if (st) return st;
    if (phasor_sample_dependent(d->kind)) return MODEM_ERR_UNSUPPORTED;
    std::memset(o, 0, sizeof *o);
    o->bits_per_symbol = bps;
    if (d->kind == MODEM_PHASOR_QAM && d->phase == 0.0f && bps % 2 == 0 && d->amplitude > 0.0f) {
        const uint32_t cs = bps / 2;
        const float ms = (float)((1u << cs) - 1);
        o->kind = MODEM_SLICER_QAM_AXIS;
        o->bits_per_carrier = cs;
        o->max_symbol = ms;
        o->inv_scale = 1.0f / (d->amplitude / ms / 2.0f);     // qam.rs:28
        return MODEM_OK;
    }
    if (!lut) return MODEM_ERR_INVALID_ARG;
    o->kind = MODEM_SLICER_NEAREST;
    o->lut = lut;
    return MODEM_OK;
}

modem_status modem_rrc_taps(uint32_t L, uint32_t sps, double beta, float* out) {
    if (!out || L == 0 || sps == 0 || !(beta >= 0.0 && beta <= 1.0)) return MODEM_ERR_INVALID_ARG;
    const double pi = 3.14159265358979323846;
    std::vector<double> h(L);
    double e = 0.0;
    for (uint32_t i = 0; i < L; ++i) {
        const double t = ((double)i - (double)(L - 1) / 2.0) / (double)sps;
        double v;
        if (t == 0.0) v = 1.0 - beta + 4.0 * beta / pi;
        else if (beta > 0.0 && std::fabs(std::fabs(4.0 * beta * t) - 1.0) < 1e-12)
            v = beta / std::sqrt(2.0) * ((1.0 + 2.0 / pi) * std::sin(pi / (4.0 * beta)) +
                                         (1.0 - 2.0 / pi) * std::cos(pi / (4.0 * beta)));
        else
            v = (std::sin(pi * t * (1.0 - beta)) + 4.0 * beta * t * std::cos(pi * t * (1.0 + beta))) /
                (pi * t * (1.0 - (4.0 * beta * t) * (4.0 * beta * t)));
        h[i] = v;
        e += v * v;
    }
    const double g = 1.0 / std::sqrt(e);
    for (uint32_t i = 0; i < L; ++i) out[i] = (float)(h[i] * g);
    return MODEM_OK;
}

// ------------------------------------------------------------------------------ TX ----
struct modem_tx {
    int device = 0;
    uint32_t bps = 0, sps = 0, ntaps = 0, K = 1;
    float w = 0.f;
    uint64_t sample = 0;
    int dtype = 0, out_mode = 0;
    float2* d_lut = nullptr;
    float* d_taps = nullptr;
    float* d_taps_q = nullptr;      // Q-rail taps when q_offset != 0
    uint32_t q_offset = 0;
    int ph_kind = 0;                // sample-dependent phasor (tx_phasor), else 0
    float ph_amp = 0.f, ph_freq = 0.f, ph_shift = 0.f, ph_max = 0.f;
    int ph_spb = 0, ph_map = 0;
    Stage scan_stage;               // per-symbol states of the scanned phasors
    Stage batch_params;             // a scan batch's parameter blocks, when this is its first handle
    float2* d_hist[2] = {nullptr, nullptr};
    uint8_t* d_carry[2] = {nullptr, nullptr};
    int hcur = 0, ccur = 0, ncarry = 0;
    int mfma_ksteps = 0;            // > 0: FIR on the matrix cores (tx_mfma)
    float* d_bfrag = nullptr;       // its split-f16 per-lane B fragments (modem_internal.h)
    std::vector<_Float16> bfrag_host;   // the same, on the host (batch compatibility check)
    float* d_luth = nullptr;        // its split-f16 LUT (re_hi, re_lo, im_hi, im_lo per entry)
    int lut_scale_exp = 0, tap_scale_exp = 0;
    int levels = 0;                 // integer-level LUT (see TxParams)
    float level_inv = 0.0f;
    uint64_t symbols = 0;           // symbols emitted so far (row-block alignment)
    Stage bits_stage, out_stage;
    ~modem_tx() {
        DeviceGuard g(device);
        for (void* p : {(void*)d_lut, (void*)d_taps, (void*)d_taps_q, (void*)d_hist[0], (void*)d_hist[1],
                        (void*)d_carry[0], (void*)d_carry[1], (void*)d_bfrag, (void*)d_luth})
            if (p) (void)hipFree(p);
    }
};

static size_t tx_sample_bytes(const modem_tx* h) {
    const size_t v = h->dtype == MODEM_DTYPE_F16 ? 2 : 4;
    return h->out_mode == MODEM_OUT_REAL ? v : 2 * v;
}

modem_status modem_tx_create(const modem_tx_desc* d, int device, modem_tx** out) {
    if (!d || !out) return MODEM_ERR_INVALID_ARG;
    *out = nullptr;
    if (d->bits_per_symbol < 1 || d->bits_per_symbol > 8) return MODEM_ERR_INVALID_ARG;
    if (d->samples_per_symbol < 1) return MODEM_ERR_INVALID_ARG;   // SymbolClock % 0 panics (data.rs:29)
    if (d->ntaps > (uint32_t)mk::kMaxTaps || (d->ntaps && !d->taps)) return MODEM_ERR_INVALID_ARG;
    if (d->dtype != MODEM_DTYPE_F32 && d->dtype != MODEM_DTYPE_F16) return MODEM_ERR_INVALID_ARG;
    if (d->out_mode < MODEM_OUT_IQ_MIXED || d->out_mode > MODEM_OUT_REAL) return MODEM_ERR_INVALID_ARG;
    // EvenOddOffset::new asserts bits_per_symbol == 2 and an even samples_per_symbol (data.rs:91-92)
    if (d->q_offset != 0 && (d->bits_per_symbol != 2 || d->samples_per_symbol % 2 != 0 ||
                             d->q_offset != d->samples_per_symbol / 2))
        return MODEM_ERR_INVALID_ARG;
    // Sample-dependent phasors (tx_phasor): sample-and-hold only; the LUT is built here.
    const modem_phasor_desc* pd = d->phasor;
    std::vector<float> plut;
    if (pd) {
        uint32_t pbps = 0;
        if (!phasor_sample_dependent(pd->kind) || phasor_bps(pd, &pbps) != MODEM_OK ||
            pbps != d->bits_per_symbol)
            return MODEM_ERR_INVALID_ARG;
        if (d->ntaps != 0) return MODEM_ERR_UNSUPPORTED;
        if (pd->kind == MODEM_PHASOR_MSK && (pd->samples_per_symbol == 0 || pd->samples_per_symbol % 2))
            return MODEM_ERR_INVALID_ARG;                                   // msk.rs:14
        if (d->q_offset && pd->kind != MODEM_PHASOR_MSK) return MODEM_ERR_UNSUPPORTED;
        if (pd->kind == MODEM_PHASOR_DCQPSK) {                              // dcqpsk.rs:23-36
            const float map[4] = {0.0f, kPi / 2.0f, 3.0f * kPi / 2.0f, kPi};
            for (int parity = 0; parity < 2; ++parity)     // even symbol count -> term + pi/4
                for (int k = 0; k < 4; ++k) {
                    const float term = parity == 0 ? map[k] + kPi / 4.0f : map[k];
                    plut.push_back(pd->amplitude * std::cos(term));         // :46-52
                    plut.push_back(pd->amplitude * std::sin(term));
                }
        }
    } else if (!d->lut) {
        return MODEM_ERR_INVALID_ARG;
    }
    if (!device_ok(device)) return MODEM_ERR_NO_DEVICE;
    DeviceGuard g(device);
    if (!g.ok) return MODEM_ERR_NO_DEVICE;
    modem_tx* h = new (std::nothrow) modem_tx;
    if (!h) return MODEM_ERR_ALLOC;
    h->device = device;
    if (pd) {
        h->ph_kind = pd->kind;
        h->ph_amp = pd->amplitude;
        h->ph_freq = pd->freq;
        h->ph_spb = (int)(pd->samples_per_symbol / 2);
        h->ph_shift = pd->shift;
        h->ph_map = pd->mfsk_map ? 1 : 0;
        h->ph_max = (float)((1u << d->bits_per_symbol) - 1u);                 // max_symbol, util.rs:13-15
    }
    h->bps = d->bits_per_symbol;
    h->sps = d->samples_per_symbol;
    h->ntaps = d->ntaps;
    h->w = d->sample_freq;
    h->sample = d->s0;
    h->dtype = d->dtype;
    h->out_mode = d->out_mode;
    h->q_offset = d->q_offset;
    // ntaps == 0: the reference's sample-and-hold == zero-stuffing + sps unit taps. A Q offset
    // D delays the Q rail: its taps are h[j - D] (length L + D).
    const uint32_t L = d->ntaps ? d->ntaps : d->samples_per_symbol;
    const uint32_t D = d->q_offset;
    h->K = (L + D + h->sps - 1) / h->sps;
    // pp[t*sps + p] = h[p + sps*t]; padded by mk::kTapPad steps of zeros so the kernels'
    // look-ahead tap loads stay in bounds.
    std::vector<float> pp((size_t)(h->K + mk::kTapPad) * h->sps, 0.0f), pq;
    auto tap = [&](uint32_t j) { return d->ntaps ? d->taps[j] : 1.0f; };
    for (uint32_t j = 0; j < L; ++j) pp[(size_t)(j / h->sps) * h->sps + j % h->sps] = tap(j);
    if (D) {
        pq.assign(pp.size(), 0.0f);
        for (uint32_t j = 0; j < L; ++j) pq[(size_t)((j + D) / h->sps) * h->sps + (j + D) % h->sps] = tap(j);
    }
    modem_status st;
    const size_t nl = pd ? std::max<size_t>(1, plut.size() / 2) : (size_t)1 << h->bps;
    const float* lut_src = pd ? plut.data() : d->lut;
    if ((st = dalloc(&h->d_lut, nl)) || (st = dalloc(&h->d_taps, pp.size())) ||
        (st = dalloc(&h->d_hist[0], h->K)) || (st = dalloc(&h->d_hist[1], h->K)) ||
        (st = dalloc(&h->d_carry[0], 8)) || (st = dalloc(&h->d_carry[1], 8)) ||
        (D && (st = dalloc(&h->d_taps_q, pq.size())))) {
        delete h;
        return st;
    }
    if ((lut_src && hipMemcpy(h->d_lut, lut_src, nl * sizeof(float2), hipMemcpyHostToDevice) != hipSuccess) ||
        hipMemcpy(h->d_taps, pp.data(), pp.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess ||
        (D && hipMemcpy(h->d_taps_q, pq.data(), pq.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess)) {
        (void)hipGetLastError();
        delete h;
        return MODEM_ERR_HIP;
    }
    // Sample-and-hold EvenOddOffset: before the first Q tick the phasor sees cur = [b0, 0]
    // (data.rs:84), i.e. the Q value of symbol index 0; it enters as the history symbol that
    // the delayed Q rail reads for n < D (its I value meets zero taps).
    // DMPSK starts from its phase (dmpsk.rs:20); MFSK / BFSK from zeros (mfsk.rs:55-56, bfsk.rs:16-17)
    if (pd && pd->kind == MODEM_PHASOR_DMPSK) {
        const float2 st0 = make_float2(pd->phase, 0.0f);
        if (hipMemcpy(h->d_hist[0], &st0, sizeof st0, hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipGetLastError();
            delete h;
            return MODEM_ERR_HIP;
        }
    }
    if (D && d->ntaps == 0 && !pd &&
        hipMemcpy(h->d_hist[0] + (h->K - 2), d->lut, sizeof(float2), hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipGetLastError();
        delete h;
        return MODEM_ERR_HIP;
    }
    // FIR path: the matrix pipe when the (sps, K) shape has an instantiated kernel, unless
    // MODEM_HIP_FIR=valu forces the packed-VALU kernel (both are parity-tested).
    const char* env = std::getenv("MODEM_HIP_FIR");
    const bool force_valu = env && std::strcmp(env, "valu") == 0;
    // Sample-and-hold (no taps) stays on the VALU kernels, which reproduce it bit for bit.
    h->mfma_ksteps = (force_valu || d->ntaps == 0 || D || pd) ? 0 : mk::tx_mfma_ksteps((int)h->sps, (int)h->K);
    if (h->mfma_ksteps > 0) {
        // Split-f16 operands of tx_mfma (modem_tx.hip). Exact power-of-two scales put the
        // maxima of the LUT and of the taps in [2^14, 2^15); both are split hi + lo =
        // rn_f16(v) + rn_f16(v - hi).
        auto scale_exp = [](float mx) {   // 0 inside [2^-3, 2^15), else into [2^14, 2^15)
            int e = 0;
            if (!(mx > 0.0f) || !std::isfinite(mx) || (mx >= 0.125f && mx < 32768.0f)) return 0;
            std::frexp(mx, &e);
            return 15 - e;
        };
        auto split = [](float v, _Float16& hi, _Float16& lo) { hi = (_Float16)v; lo = (_Float16)(v - (float)hi); };
        float lmax = 0.0f, tmax = 0.0f;
        for (size_t k = 0; k < 2 * nl; ++k) lmax = std::max(lmax, std::fabs(d->lut[k]));
        for (uint32_t k = 0; k < d->ntaps; ++k) tmax = std::max(tmax, std::fabs(d->taps[k]));
        // Integer levels: every component v = q * s, q an integer with |q| <= 2048 (exact f16),
        // s the smallest nonzero |component|. Then A = q exactly and s moves into the taps.
        double smin = 0.0;
        for (size_t k = 0; k < 2 * nl; ++k) {
            const double a = std::fabs((double)d->lut[k]);
            if (a > 0.0 && (smin == 0.0 || a < smin)) smin = a;
        }
        bool levels = smin > 0.0;
        for (size_t k = 0; levels && k < 2 * nl; ++k) {
            const double q = (double)d->lut[k] / smin, r = std::nearbyint(q);
            levels = std::fabs(r) <= 2048.0 && std::fabs(q - r) <= 1e-6 * std::max(1.0, std::fabs(q));
        }
        h->levels = levels ? 1 : 0;
        h->level_inv = levels ? (float)(1.0 / smin) : 0.0f;
        const double tscale = levels ? smin : 1.0;           // folded into the taps
        tmax = (float)(tmax * tscale);
        h->lut_scale_exp = levels ? 0 : scale_exp(lmax);
        h->tap_scale_exp = scale_exp(tmax);
        std::vector<_Float16> lh(4 * nl);
        for (size_t k = 0; k < nl; ++k) {
            if (levels) {
                lh[4 * k] = (_Float16)std::nearbyint((double)d->lut[2 * k] / smin);
                lh[4 * k + 2] = (_Float16)std::nearbyint((double)d->lut[2 * k + 1] / smin);
                lh[4 * k + 1] = lh[4 * k + 3] = (_Float16)0.0f;
                continue;
            }
            split(std::ldexp(d->lut[2 * k], h->lut_scale_exp), lh[4 * k], lh[4 * k + 1]);
            split(std::ldexp(d->lut[2 * k + 1], h->lut_scale_exp), lh[4 * k + 2], lh[4 * k + 3]);
        }
        // B[o][j] = h[p + sps*(c + PRE - o)], j = sps*c + p: lane l holds, for k-step s, the 8
        // window offsets o = 32s + 8(l >> 4) + jj of column j = l & 15, hi then lo.
        const int nks = h->mfma_ksteps, sps = (int)h->sps, SB = 16 / sps, PRE = 32 * nks - SB;
        std::vector<_Float16> bf((size_t)nks * 2 * 64 * 8, (_Float16)0.0f);
        for (int s2 = 0; s2 < nks; ++s2)
            for (int l = 0; l < 64; ++l)
                for (int jj = 0; jj < 8; ++jj) {
                    const int o = 32 * s2 + 8 * (l >> 4) + jj, j = l & 15, c = j / sps, ph = j % sps;
                    const int t = c + PRE - o;
                    const float v = (t >= 0 && t < (int)h->K)
                        ? std::ldexp((float)((double)pp[(size_t)t * sps + ph] * tscale), h->tap_scale_exp) : 0.0f;
                    split(v, bf[(((size_t)s2 * 2) * 64 + l) * 8 + jj], bf[(((size_t)s2 * 2 + 1) * 64 + l) * 8 + jj]);
                }
        const size_t nb = (bf.size() * sizeof(_Float16) + sizeof(float) - 1) / sizeof(float);
        const size_t nlh = (lh.size() * sizeof(_Float16) + sizeof(float) - 1) / sizeof(float);
        if ((st = dalloc(&h->d_bfrag, nb)) || (st = dalloc(&h->d_luth, nlh))) { delete h; return st; }
        h->bfrag_host = bf;
        if (hipMemcpy(h->d_bfrag, bf.data(), bf.size() * sizeof(_Float16), hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(h->d_luth, lh.data(), lh.size() * sizeof(_Float16), hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipGetLastError();
            delete h;
            return MODEM_ERR_HIP;
        }
    }
    *out = h;
    return MODEM_OK;
}

// Non-temporal TX stores for large launches. A launch writing more than the Infinity Cache
// holds (256 MiB on MI355X) streams its samples through it to HBM anyway, and its dirty lines
// are then written back while the RX reads the buffer. Such a launch (over 192 MiB: C5, 512
// MiB) stores its samples non-temporally, straight to HBM. In-tree A/B of this host switch
// (profiles/r03_tx_nt.txt, bench legs): C5 chain 280.9 -> 268.5 us, TX alone 135 -> 109 us,
// the RX in the chain 145.5 -> 159.5 us (it now reads everything from HBM); C4 chain 121 ->
// 116.6 us. (The earlier compile-time all-NT build measured C5 chain 273.4 -> 257.9 us on
// another box; keeping the last 128 MiB cacheable, 261.4.) A single-channel launch of at most
// the Infinity Cache's size (C5 f16: 256 MiB) stores only its first half non-temporally: the
// RX, walking its tiles top-down, then finds the second half in the cache (chain 182.6 ->
// 178.3-179.2 us, profiles/r04_tx_nt.txt; the same split for C5 f32 and for C4's 8-channel
// batch was slower: 265 vs 261 us, 125.8 vs 120 us). Smaller launches (C3: 128 MiB, whose RX
// re-reads it from the cache) keep the default policy. MODEM_TX_NT=0 turns it off (A/B),
// MODEM_TX_NT=1 stores every large launch's samples non-temporally.
// `launch_bytes`: the whole launch's output (every channel of a batch); returns nt_below.
static int64_t tx_nt_below(int64_t nsamp, uint64_t launch_bytes, bool single) {
    static const int mode = [] { const char* e = std::getenv("MODEM_TX_NT"); return e ? std::atoi(e) : 2; }();
    constexpr uint64_t kMin = 192ull << 20, kCache = 256ull << 20;
    if (mode == 0 || launch_bytes <= kMin || nsamp <= 0) return 0;
    // the cacheable second half pays only because the RX reads it first (mk::kRxTilesTopDown)
    return mode == 2 && single && mk::kRxTilesTopDown && launch_bytes <= kCache ? nsamp / 2 : nsamp;
}

// Kernel parameters of one TX call on device buffers (dbits, dout); see tx_run.
static void tx_fill(const modem_tx* h, const uint8_t* dbits, size_t nbits, bool flush, void* dout,
                    int64_t nsym, int ncarry_new, size_t nsamp, mk::TxParams& p) {
    p.bits = dbits;
    p.carry = h->d_carry[h->ccur];
    p.carry_new = h->d_carry[h->ccur ^ 1];
    p.hist = h->d_hist[h->hcur];
    p.hist_new = h->d_hist[h->hcur ^ 1];
    p.lut = h->d_lut;
    p.taps = h->d_taps;
    p.taps_q = h->d_taps_q;
    p.out = dout;
    p.nt_below = tx_nt_below((int64_t)nsamp, (uint64_t)nsamp * tx_sample_bytes(h), true);
    p.s0 = h->sample;
    p.nsym = nsym;
    p.nsym_valid = flush ? 0 : nsym;
    p.nbits = (int64_t)nbits;
    p.ncarry = h->ncarry;
    p.ncarry_new = ncarry_new;
    p.update_carry = flush ? 0 : 1;
    p.bps = (int)h->bps;
    p.sps = (int)h->sps;
    p.K = (int)h->K;
    p.fast_bits = (h->ncarry == 0 && (h->bps == 1 || h->bps == 2 || h->bps == 4 || h->bps == 8) &&
                   ((uintptr_t)dbits % h->bps) == 0) ? 1 : 0;
    p.exact_idx = (h->sample + nsamp) <= (1ull << 53) ? 1 : 0;
    p.idx46 = (h->sample + nsamp + 256) < (1ull << 46) ? 1 : 0;
    p.w = h->w;
    p.lut_h = h->d_luth;
    p.lut_scale_exp = h->lut_scale_exp;
    p.tap_scale_exp = h->tap_scale_exp;
    p.levels = h->levels;
    p.level_inv = h->level_inv;
    const uint32_t sb = (h->sps <= 16 && 16 % h->sps == 0) ? 16 / h->sps : 1;   // symbols per row-block
    p.lead = (int)(h->symbols % sb);
    p.ph_kind = h->ph_kind;
    p.sym0 = h->symbols;
    p.ph_amp = h->ph_amp;
    p.ph_freq = h->ph_freq;
    p.ph_spb = h->ph_spb;
    p.q_off = (int)h->q_offset;
    p.ph_shift = h->ph_shift;
    p.ph_map = h->ph_map;
    p.ph_max = h->ph_max;
}

// The handle's state after a TX call (the kernel wrote the other history / carry buffers).
static void tx_advance(modem_tx* h, bool flush, int64_t nsym, int ncarry_new, size_t nsamp) {
    h->hcur ^= 1;
    if (!flush) { h->ccur ^= 1; h->ncarry = ncarry_new; }
    h->sample += nsamp;
    h->symbols += (uint64_t)nsym;
}

// The kernel launch of one TX call on device buffers and the handle's state update.
static modem_status tx_launch(modem_tx* h, const uint8_t* dbits, size_t nbits, bool flush, void* dout, int64_t nsym,
                              int ncarry_new, size_t nsamp, hipStream_t s) {
    modem_status st;
    mk::TxParams p{};
    tx_fill(h, dbits, nbits, flush, dout, nsym, ncarry_new, nsamp, p);
    p.scan = nullptr;
    if (phasor_scanned(h->ph_kind)) {
        if ((st = h->scan_stage.ensure((size_t)std::max<int64_t>(nsym, 1) * sizeof(float2)))) return st;
        p.scan = static_cast<float2*>(h->scan_stage.p);
    }
    if (h->ph_kind)
        HIP_TRY(mk::launch_tx_phasor(p, h->dtype, h->out_mode, s));
    else if (h->mfma_ksteps > 0)
        HIP_TRY(mk::launch_tx_mfma(p, (int)h->sps, h->mfma_ksteps, h->d_bfrag, h->dtype, h->out_mode, s));
    else
        HIP_TRY(mk::launch_tx(p, (int)h->sps, h->dtype, h->out_mode, s));
    tx_advance(h, flush, nsym, ncarry_new, nsamp);
    return MODEM_OK;
}

static modem_status tx_run(modem_tx* h, const uint8_t* bits, size_t nbits, bool flush, void* out,
                           size_t cap, size_t* produced, hipStream_t s) {
    if (!h || !produced || (nbits && !bits)) return MODEM_ERR_INVALID_ARG;
    *produced = 0;
    const uint64_t total = (uint64_t)h->ncarry + nbits;
    const int64_t nsym = flush ? (int64_t)((h->ntaps ? h->ntaps - 1 + h->q_offset : 0) + h->sps - 1) / h->sps
                               : (int64_t)(total / h->bps);
    const int ncarry_new = flush ? h->ncarry : (int)(total - (uint64_t)nsym * h->bps);
    const size_t nsamp = (size_t)nsym * h->sps;
    if (nsamp > cap) return MODEM_ERR_CAPACITY;
    if (nsamp && !out) return MODEM_ERR_INVALID_ARG;
    const PtrKind kb = nbits ? ptr_kind(bits, h->device) : PTR_DEVICE;
    const PtrKind ko = nsamp ? ptr_kind(out, h->device) : PTR_DEVICE;
    if (kb == PTR_FOREIGN || ko == PTR_FOREIGN) return MODEM_ERR_INVALID_ARG;
    DeviceGuard g(h->device);
    if (!g.ok) return MODEM_ERR_NO_DEVICE;
    modem_status st;
    const uint8_t* dbits = bits;
    if (kb == PTR_HOST) {
        if ((st = h->bits_stage.ensure(nbits))) return st;
        HIP_TRY(hipMemcpyAsync(h->bits_stage.p, bits, nbits, hipMemcpyHostToDevice, s));
        dbits = static_cast<const uint8_t*>(h->bits_stage.p);
    }
    const bool host_out = ko == PTR_HOST;
    void* dout = out;
    if (host_out) {
        if ((st = h->out_stage.ensure(nsamp * tx_sample_bytes(h)))) return st;
        dout = h->out_stage.p;
    }
    if ((st = tx_launch(h, dbits, nbits, flush, dout, nsym, ncarry_new, nsamp, s))) return st;
    if (host_out) {
        HIP_TRY(hipMemcpyAsync(out, dout, nsamp * tx_sample_bytes(h), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    } else if (nbits && dbits != bits) {
        HIP_TRY(hipStreamSynchronize(s));   // host bits staged: keep the caller's view simple
    }
    *produced = nsamp;
    return MODEM_OK;
}

modem_status modem_tx_process(modem_tx* h, const uint8_t* bits, size_t nbits, void* out, size_t cap,
                              size_t* produced, void* stream) {
    return tx_run(h, bits, nbits, false, out, cap, produced, (hipStream_t)stream);
}
modem_status modem_tx_flush(modem_tx* h, void* out, size_t cap, size_t* produced, void* stream) {
    return tx_run(h, nullptr, 0, true, out, cap, produced, (hipStream_t)stream);
}
// Channels of one scanned phasor kind (DMPSK / MFSK / BFSK; modem_tx_process_batch): their serial
// symbol-state scans run as one launch, one lane per channel (tx_scan_batch: each channel's
// states bit for bit those of its single call), then each channel's sample kernel. Every buffer is
// device memory; the handles are distinct and share a device.
static modem_status tx_scan_batch_run(modem_tx* const* hs, size_t nch, const uint8_t* const* bits,
                                      const size_t* nbits, void* const* outs, const size_t* caps, size_t* produced,
                                      hipStream_t s) {
    std::vector<int64_t> nsym(nch);
    std::vector<int> ncarry_new(nch);
    for (size_t c = 0; c < nch; ++c) {        // every channel's size first: an error leaves the handles untouched
        const modem_tx* h = hs[c];
        const uint64_t total = (uint64_t)h->ncarry + nbits[c];
        nsym[c] = (int64_t)(total / h->bps);
        ncarry_new[c] = (int)(total - (uint64_t)nsym[c] * h->bps);
        if ((size_t)nsym[c] * h->sps > caps[c]) return MODEM_ERR_CAPACITY;
    }
    DeviceGuard g(hs[0]->device);
    if (!g.ok) return MODEM_ERR_NO_DEVICE;
    modem_status st;
    std::vector<mk::TxParams> ps(nch);
    for (size_t c = 0; c < nch; ++c) {
        modem_tx* h = hs[c];
        if ((st = h->scan_stage.ensure((size_t)std::max<int64_t>(nsym[c], 1) * sizeof(float2)))) return st;
        tx_fill(h, bits[c], nbits[c], false, outs[c], nsym[c], ncarry_new[c], (size_t)nsym[c] * h->sps, ps[c]);
        ps[c].scan = static_cast<float2*>(h->scan_stage.p);
    }
    if ((st = hs[0]->batch_params.ensure(nch * sizeof(mk::TxParams)))) return st;
    // (from pageable host memory: synchronous, so `ps` may go when the call returns)
    HIP_TRY(hipMemcpyAsync(hs[0]->batch_params.p, ps.data(), nch * sizeof(mk::TxParams), hipMemcpyHostToDevice, s));
    HIP_TRY(mk::launch_tx_scan_batch(static_cast<const mk::TxParams*>(hs[0]->batch_params.p), (int)nch,
                                      hs[0]->ph_kind, s));
    for (size_t c = 0; c < nch; ++c) {
        modem_tx* h = hs[c];
        HIP_TRY(mk::launch_tx_phasor(ps[c], h->dtype, h->out_mode, s, true));
        tx_advance(h, false, nsym[c], ncarry_new[c], (size_t)nsym[c] * h->sps);
        produced[c] = (size_t)nsym[c] * h->sps;
    }
    return MODEM_OK;
}

// One launch for several channels (independent channel streams). Equivalent to
// modem_tx_process(hs[c], bits[c], nbits[c], outs[c], caps[c], &produced[c], stream) for
// c = 0 .. nch-1 in order; fused into one launch per kBatchMax channels when every handle
// shares the matrix-core configuration (sps, taps, bps, f32/f16 mixed I/Q output, device)
// and all buffers are device memory, otherwise run one call at a time.
modem_status modem_tx_process_batch(modem_tx* const* hs, size_t nch, const uint8_t* const* bits,
                                    const size_t* nbits, void* const* outs, const size_t* caps,
                                    size_t* produced, void* stream) {
    if (nch == 0) return MODEM_OK;
    if (!hs || !bits || !nbits || !outs || !caps || !produced) return MODEM_ERR_INVALID_ARG;
    const hipStream_t s = (hipStream_t)stream;
    for (size_t c = 0; c < nch; ++c)    // an error leaves every handle untouched
        if (hs[c] && ((nbits[c] && foreign_ptr(bits[c], hs[c]->device)) || foreign_ptr(outs[c], hs[c]->device)))
            return MODEM_ERR_INVALID_ARG;
    bool scan = nch >= 2 && hs[0] != nullptr && phasor_scanned(hs[0]->ph_kind);
    for (size_t c = 0; scan && c < nch; ++c) {
        const modem_tx* h = hs[c];
        scan = h && h->device == hs[0]->device && h->ph_kind == hs[0]->ph_kind &&
               (nbits[c] == 0 || (bits[c] && is_device_ptr(bits[c]))) && outs[c] && is_device_ptr(outs[c]);
        for (size_t e = 0; scan && e < c; ++e) scan = hs[e] != h;      // a handle at most once
    }
    if (scan) {
        for (size_t c = 0; c < nch; ++c) produced[c] = 0;
        return tx_scan_batch_run(hs, nch, bits, nbits, outs, caps, produced, s);
    }
    bool fuse = nch >= 2 && hs[0] != nullptr;
    for (size_t c = 0; fuse && c < nch; ++c) {
        const modem_tx* h = hs[c];
        const modem_tx* h0 = hs[0];
        fuse = h && h->device == h0->device && h->ph_kind == 0 && h->mfma_ksteps > 0 &&
               h->mfma_ksteps == h0->mfma_ksteps && h->out_mode == MODEM_OUT_IQ_MIXED && h->dtype == h0->dtype &&
               h->sps == h0->sps && h->bps == h0->bps && h->ntaps == h0->ntaps && h->q_offset == 0 &&
               h->bfrag_host == h0->bfrag_host && (nbits[c] == 0 || (bits[c] && is_device_ptr(bits[c]))) &&
               outs[c] && is_device_ptr(outs[c]);
        for (size_t e = 0; fuse && e < c; ++e) fuse = hs[e] != h;      // a handle at most once
    }
    if (!fuse) {
        for (size_t c = 0; c < nch; ++c) {
            const modem_status st = tx_run(hs[c], bits[c], nbits[c], false, outs[c], caps[c], &produced[c], s);
            if (st != MODEM_OK) return st;
        }
        return MODEM_OK;
    }
    for (size_t c = 0; c < nch; ++c) produced[c] = 0;
    // check every channel first: an error leaves all handles untouched
    std::vector<int64_t> nsym(nch);
    std::vector<int> ncarry_new(nch);
    for (size_t c = 0; c < nch; ++c) {
        const modem_tx* h = hs[c];
        const uint64_t total = (uint64_t)h->ncarry + nbits[c];
        nsym[c] = (int64_t)(total / h->bps);
        ncarry_new[c] = (int)(total - (uint64_t)nsym[c] * h->bps);
        if ((size_t)nsym[c] * h->sps > caps[c]) return MODEM_ERR_CAPACITY;
    }
    DeviceGuard g(hs[0]->device);
    if (!g.ok) return MODEM_ERR_NO_DEVICE;
    for (size_t c0 = 0; c0 < nch; c0 += mk::kBatchMax) {
        mk::TxBatch b{};
        b.nch = (int32_t)std::min<size_t>(mk::kBatchMax, nch - c0);
        for (int i = 0; i < b.nch; ++i) {
            const size_t c = c0 + (size_t)i;
            tx_fill(hs[c], bits[c], nbits[c], false, outs[c], nsym[c], ncarry_new[c], (size_t)nsym[c] * hs[c]->sps, b.p[i]);
        }
        uint64_t launch_bytes = 0;          // the non-temporal split over the whole launch
        for (int i = 0; i < b.nch; ++i)
            launch_bytes += (uint64_t)nsym[c0 + i] * hs[c0 + i]->sps * tx_sample_bytes(hs[c0 + i]);
        for (int i = 0; i < b.nch; ++i)
            b.p[i].nt_below = tx_nt_below(nsym[c0 + i] * (int64_t)hs[c0 + i]->sps, launch_bytes, false);
        HIP_TRY(mk::launch_tx_mfma_batch(b, (int)hs[0]->sps, hs[0]->mfma_ksteps, hs[0]->d_bfrag, hs[0]->dtype, s));
        for (int i = 0; i < b.nch; ++i) {
            const size_t c = c0 + (size_t)i;
            modem_tx* h = hs[c];
            h->hcur ^= 1;
            h->ccur ^= 1;
            h->ncarry = ncarry_new[c];
            h->sample += (uint64_t)nsym[c] * h->sps;
            h->symbols += (uint64_t)nsym[c];
            produced[c] = (size_t)nsym[c] * h->sps;
        }
    }
    return MODEM_OK;
}
uint64_t modem_tx_sample(const modem_tx* h) { return h ? h->sample : 0; }
modem_status modem_tx_destroy(modem_tx* h) { delete h; return MODEM_OK; }

// ------------------------------------------------------------------------------ RX ----
struct modem_rx {
    int device = 0;
    uint32_t ntaps = 0, decim = 1, D = 0, K = 1, HL = 0;
    int mix = 0, in_dtype = 0, out_dtype = 0;
    float w = 0.f;
    uint64_t c0 = 0;
    float phase_offset = 0.f;       // PLL offset (demodulator.rs:50)
    int64_t consumed = 0;          // stream samples processed
    modem_slicer_desc slicer{};
    int mfma_ksteps = 0;            // > 0: matched filter on the matrix pipe (rx_mfma)
    float* d_bfrag = nullptr;       // its split-f16 tap tables (modem_internal.h)
    std::vector<_Float16> bfrag_host;   // the same, on the host (batch compatibility check)
    int tap_scale_exp = 0;          // the tables hold h * 2^tap_scale_exp
    float* d_taps = nullptr;
    float2* d_slut = nullptr;
    void* d_hist[2] = {nullptr, nullptr};
    int* d_ka = nullptr;            // rx_mfma staging-exponent prediction, double-buffered like d_hist
    void* d_zeros = nullptr;
    int hcur = 0;
    Stage in_stage, iq_stage, sym_stage;
    ~modem_rx() {
        DeviceGuard g(device);
        for (void* p : {(void*)d_taps, (void*)d_slut, d_hist[0], d_hist[1], d_zeros, (void*)d_bfrag, (void*)d_ka})
            if (p) (void)hipFree(p);
    }
};

static size_t rx_in_bytes(const modem_rx* h) {
    return h->in_dtype == MODEM_DTYPE_I16 ? 2 : h->in_dtype == MODEM_DTYPE_F16 ? 4 : 8;
}
static size_t rx_out_bytes(const modem_rx* h) { return h->out_dtype == MODEM_DTYPE_F16 ? 4 : 8; }

modem_status modem_rx_create(const modem_rx_desc* d, int device, modem_rx** out) {
    if (!d || !out) return MODEM_ERR_INVALID_ARG;
    *out = nullptr;
    if (d->ntaps < 1 || d->ntaps > (uint32_t)mk::kMaxTaps || !d->taps) return MODEM_ERR_INVALID_ARG;
    if (d->decim < 1) return MODEM_ERR_INVALID_ARG;
    if (d->mix != MODEM_MIX_COMPLEX && d->mix != MODEM_MIX_REFERENCE_REAL && d->mix != MODEM_MIX_REFERENCE_REAL_EXACT)
        return MODEM_ERR_INVALID_ARG;
    if ((d->in_dtype != MODEM_DTYPE_F32 && d->in_dtype != MODEM_DTYPE_F16 && d->in_dtype != MODEM_DTYPE_I16) ||
        (d->out_dtype != MODEM_DTYPE_F32 && d->out_dtype != MODEM_DTYPE_F16)) return MODEM_ERR_INVALID_ARG;
    // real i16 input: the exact reference demodulator only (the complex kernels read I/Q pairs)
    if (d->in_dtype == MODEM_DTYPE_I16 && d->mix != MODEM_MIX_REFERENCE_REAL_EXACT) return MODEM_ERR_UNSUPPORTED;
    const modem_slicer_desc& sl = d->slicer;
    if (sl.kind == MODEM_SLICER_NEAREST && (sl.bits_per_symbol < 1 || sl.bits_per_symbol > 8 || !sl.lut))
        return MODEM_ERR_INVALID_ARG;
    if (sl.kind == MODEM_SLICER_QAM_AXIS && (sl.bits_per_carrier < 1 || sl.bits_per_carrier > 4))
        return MODEM_ERR_INVALID_ARG;
    if (sl.kind < MODEM_SLICER_NONE || sl.kind > MODEM_SLICER_QAM_AXIS) return MODEM_ERR_INVALID_ARG;
    if (!device_ok(device)) return MODEM_ERR_NO_DEVICE;
    DeviceGuard g(device);
    if (!g.ok) return MODEM_ERR_NO_DEVICE;
    modem_rx* h = new (std::nothrow) modem_rx;
    if (!h) return MODEM_ERR_ALLOC;
    h->device = device;
    h->ntaps = d->ntaps;
    h->decim = d->decim;
    h->D = d->decim_offset;
    h->K = (d->ntaps + d->decim - 1) / d->decim;
    h->HL = h->K * h->decim - 1;
    h->mix = d->mix;
    h->in_dtype = d->in_dtype;
    h->out_dtype = d->out_dtype;
    h->w = d->sample_freq;
    h->c0 = d->s0;
    h->phase_offset = d->phase_offset;
    h->slicer = sl;
    h->slicer.lut = nullptr;
    // pp[b*K + t] = h[b + decim*t], padded for the kernels' look-ahead tap loads
    std::vector<float> pp((size_t)h->K * h->decim + mk::kTapPad, 0.0f);
    for (uint32_t j = 0; j < d->ntaps; ++j) pp[(size_t)(j % h->decim) * h->K + j / h->decim] = d->taps[j];
    const size_t esz = rx_in_bytes(h);
    modem_status st;
    uint8_t *h0 = nullptr, *h1 = nullptr, *z = nullptr;
    if ((st = dalloc(&h->d_taps, pp.size())) || (st = dalloc(&h->d_slut, 256)) ||
        (st = dalloc(&h0, (h->HL + 1) * esz)) || (st = dalloc(&h1, (h->HL + 1) * esz)) ||
        (st = dalloc(&z, (size_t)(h->ntaps) * esz))) {
        h->d_hist[0] = h0; h->d_hist[1] = h1; h->d_zeros = z;
        delete h;
        return st;
    }
    h->d_hist[0] = h0; h->d_hist[1] = h1; h->d_zeros = z;
    const int ka_none[2] = {INT32_MIN, INT32_MIN};
    if ((st = dalloc(&h->d_ka, 2))) { delete h; return st; }
    if (hipMemcpy(h->d_taps, pp.data(), pp.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(h->d_ka, ka_none, sizeof ka_none, hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipGetLastError(); delete h; return MODEM_ERR_HIP;
    }
    if (sl.kind == MODEM_SLICER_NEAREST &&
        hipMemcpy(h->d_slut, sl.lut, ((size_t)2 << sl.bits_per_symbol) * sizeof(float),
                  hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipGetLastError(); delete h; return MODEM_ERR_HIP;
    }
    const char* env = std::getenv("MODEM_HIP_FIR");
    const bool force_valu = env && std::strcmp(env, "valu") == 0;
    const bool exact = h->mix == MODEM_MIX_REFERENCE_REAL_EXACT;
    h->mfma_ksteps = force_valu || exact ? 0 : mk::rx_mfma_ksteps((int)h->decim, (int)h->ntaps);
    if (h->mfma_ksteps > 0) {
        // Split-f16 tap tables of rx_mfma (modem_rx.hip): the reversed taps T[x] = h[W-1-x]
        // scaled by 2^kb (exact; 0 when max |h| is in [2^-3, 2^15), else into [2^14, 2^15)), as f16
        // hi then lo = rn_f16(v - hi), in NC copies shifted by gcd(decim, 8) so that every
        // lane's 8-tap read is 16-B aligned.
        const int nks = h->mfma_ksteps, W = 32 * nks, dec = (int)h->decim;
        const int nc = mk::rx_mfma_table_copies(dec), tb = mk::rx_mfma_table_len(dec, nks), gq = 8 / nc;
        float hmax = 0.0f;
        for (uint32_t k = 0; k < h->ntaps; ++k) hmax = std::max(hmax, std::fabs(d->taps[k]));
        int kb = 0;   // 0 inside [2^-3, 2^15), else into [2^14, 2^15)
        if (hmax > 0.0f && std::isfinite(hmax) && !(hmax >= 0.125f && hmax < 32768.0f)) {
            int e;
            std::frexp(hmax, &e);
            kb = 15 - e;
        }
        h->tap_scale_exp = kb;
        std::vector<_Float16> tab((size_t)nc * 2 * tb, (_Float16)0.0f);
        for (int c = 0; c < nc; ++c)
            for (int y = 0; y < tb; ++y) {
                const int u = W - 1 - (y + c * gq);
                const float v = (u >= 0 && u < (int)h->ntaps) ? std::ldexp(d->taps[u], kb) : 0.0f;
                const _Float16 hi = (_Float16)v;
                tab[((size_t)c * 2) * tb + y] = hi;
                tab[((size_t)c * 2 + 1) * tb + y] = (_Float16)(v - (float)hi);
            }
        const size_t nfl = (tab.size() * sizeof(_Float16) + sizeof(float) - 1) / sizeof(float);
        if ((st = dalloc(&h->d_bfrag, nfl))) { delete h; return st; }
        h->bfrag_host = tab;
        if (hipMemcpy(h->d_bfrag, tab.data(), tab.size() * sizeof(_Float16), hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipGetLastError(); delete h; return MODEM_ERR_HIP;
        }
    }
    *out = h;
    return MODEM_OK;
}

// Kept instants n = k*decim + D with n in [a, b): first k and count.
static void rx_range(int64_t a, int64_t b, int64_t decim, int64_t D, int64_t* k0, int64_t* cnt) {
    auto first_at_or_after = [&](int64_t n) -> int64_t {
        return n <= D ? 0 : (n - D + decim - 1) / decim;
    };
    *k0 = first_at_or_after(a);
    const int64_t k1 = first_at_or_after(b);
    *cnt = k1 > *k0 ? k1 - *k0 : 0;
}

// Kernel parameters of one RX call on device buffers; see rx_run.
static void rx_fill(const modem_rx* h, const void* din, size_t n, void* diq, uint8_t* dsym, int64_t k_first,
                    int64_t nout, mk::RxParams& p) {
    p.x = din;
    p.hist = h->d_hist[h->hcur];
    p.hist_new = h->d_hist[h->hcur ^ 1];
    p.out_iq = nout ? diq : nullptr;
    p.out_sym = nout ? dsym : nullptr;
    p.taps = h->d_taps;
    p.slut = h->d_slut;
    p.N = (int64_t)n;
    p.n_start = h->consumed;
    p.c0 = h->c0;
    p.k_first = k_first;
    p.nout = nout;
    p.K = (int)h->K;
    p.L = (int)h->ntaps;
    p.HL = (int)h->HL;
    p.D = (int)h->D;
    p.decim = (int)h->decim;
    p.x_aligned16 = ((uintptr_t)din % 16) == 0 ? 1 : 0;
    p.phase_offset = h->phase_offset;
    p.exact_idx = (h->c0 + (uint64_t)h->consumed + n + (uint64_t)h->HL) <= (1ull << 53) ? 1 : 0;
    p.idx46 = (h->c0 + (uint64_t)h->consumed + n + (uint64_t)h->HL + 65536) < (1ull << 46) ? 1 : 0;
    p.ka_in = h->d_ka + h->hcur;
    p.ka_out = h->d_ka + (h->hcur ^ 1);
    p.slicer_kind = h->slicer.kind;
    p.bps = (int)h->slicer.bits_per_symbol;
    p.bits_per_carrier = (int)h->slicer.bits_per_carrier;
    p.inv_scale = h->slicer.inv_scale;
    p.max_symbol = h->slicer.max_symbol;
    p.w = h->w;
    p.tap_scale_exp = h->tap_scale_exp;
}

// The handle's state after an RX call (the kernel wrote the other history / ka slot).
static void rx_advance(modem_rx* h, size_t n) {
    h->hcur ^= 1;
    h->consumed += (int64_t)n;
}

// The kernel launch of one RX call on device buffers and the handle's state update.
static modem_status rx_launch(modem_rx* h, const void* din, size_t n, void* diq, uint8_t* dsym, int64_t k_first,
                              int64_t nout, hipStream_t s) {
    mk::RxParams p{};
    rx_fill(h, din, n, diq, dsym, k_first, nout, p);
    if (h->mfma_ksteps > 0) {
        HIP_TRY(mk::launch_rx_mfma(p, (int)h->decim, h->mfma_ksteps, h->d_bfrag, h->in_dtype, h->out_dtype,
                                   h->mix, s));
    } else
        HIP_TRY(mk::launch_rx(p, (int)h->decim, h->in_dtype, h->out_dtype, h->mix, s));
    rx_advance(h, n);
    return MODEM_OK;
}

static modem_status rx_run(modem_rx* h, const void* in, size_t n, bool zeros, void* out_iq,
                           uint8_t* out_sym, size_t cap, size_t* produced, hipStream_t s) {
    if (!h || !produced || (n && !in && !zeros)) return MODEM_ERR_INVALID_ARG;
    *produced = 0;
    int64_t k_first, nout;
    rx_range(h->consumed, h->consumed + (int64_t)n, h->decim, h->D, &k_first, &nout);
    if ((size_t)nout > cap) return MODEM_ERR_CAPACITY;
    const PtrKind ki = n && !zeros ? ptr_kind(in, h->device) : PTR_DEVICE;
    const PtrKind kq = nout && out_iq ? ptr_kind(out_iq, h->device) : PTR_DEVICE;
    const PtrKind ks = nout && out_sym ? ptr_kind(out_sym, h->device) : PTR_DEVICE;
    if (ki == PTR_FOREIGN || kq == PTR_FOREIGN || ks == PTR_FOREIGN) return MODEM_ERR_INVALID_ARG;
    DeviceGuard g(h->device);
    if (!g.ok) return MODEM_ERR_NO_DEVICE;
    modem_status st;
    const void* din = zeros ? h->d_zeros : in;
    if (ki == PTR_HOST) {
        if ((st = h->in_stage.ensure(n * rx_in_bytes(h)))) return st;
        HIP_TRY(hipMemcpyAsync(h->in_stage.p, in, n * rx_in_bytes(h), hipMemcpyHostToDevice, s));
        din = h->in_stage.p;
    }
    const bool host_iq = kq == PTR_HOST;
    const bool host_sym = ks == PTR_HOST;
    void* diq = out_iq;
    uint8_t* dsym = out_sym;
    if (host_iq) {
        if ((st = h->iq_stage.ensure((size_t)nout * rx_out_bytes(h)))) return st;
        diq = h->iq_stage.p;
    }
    if (host_sym) {
        if ((st = h->sym_stage.ensure((size_t)nout))) return st;
        dsym = static_cast<uint8_t*>(h->sym_stage.p);
    }
    if ((st = rx_launch(h, din, n, diq, dsym, k_first, nout, s))) return st;
    if (host_iq) HIP_TRY(hipMemcpyAsync(out_iq, diq, (size_t)nout * rx_out_bytes(h), hipMemcpyDeviceToHost, s));
    if (host_sym) HIP_TRY(hipMemcpyAsync(out_sym, dsym, (size_t)nout, hipMemcpyDeviceToHost, s));
    if (host_iq || host_sym || din == h->in_stage.p) HIP_TRY(hipStreamSynchronize(s));
    *produced = (size_t)nout;
    return MODEM_OK;
}

modem_status modem_rx_process(modem_rx* h, const void* in, size_t n, void* out_iq, uint8_t* out_sym,
                              size_t cap, size_t* produced, void* stream) {
    return rx_run(h, in, n, false, out_iq, out_sym, cap, produced, (hipStream_t)stream);
}
modem_status modem_rx_flush(modem_rx* h, void* out_iq, uint8_t* out_sym, size_t cap, size_t* produced,
                            void* stream) {
    if (!h) return MODEM_ERR_INVALID_ARG;
    return rx_run(h, nullptr, h->ntaps - 1, true, out_iq, out_sym, cap, produced, (hipStream_t)stream);
}
// One launch for several channels; equivalent to modem_rx_process on each in order. Fused
// per kBatchMax channels when every handle shares the matrix-core configuration (decim,
// taps, complex mix, one I/Q dtype in and out, device) and all buffers are device memory.
modem_status modem_rx_process_batch(modem_rx* const* hs, size_t nch, const void* const* ins, const size_t* ns,
                                    void* const* out_iq, uint8_t* const* out_sym, const size_t* caps,
                                    size_t* produced, void* stream) {
    if (nch == 0) return MODEM_OK;
    if (!hs || !ins || !ns || !out_iq || !out_sym || !caps || !produced) return MODEM_ERR_INVALID_ARG;
    const hipStream_t s = (hipStream_t)stream;
    for (size_t c = 0; c < nch; ++c)
        if (hs[c] && ((ns[c] && foreign_ptr(ins[c], hs[c]->device)) || foreign_ptr(out_iq[c], hs[c]->device) ||
                      foreign_ptr(out_sym[c], hs[c]->device)))
            return MODEM_ERR_INVALID_ARG;
    bool fuse = nch >= 2 && hs[0] != nullptr;
    for (size_t c = 0; fuse && c < nch; ++c) {
        const modem_rx* h = hs[c];
        const modem_rx* h0 = hs[0];
        fuse = h && h->device == h0->device && h->mfma_ksteps > 0 && h->mfma_ksteps == h0->mfma_ksteps &&
               h->mix == MODEM_MIX_COMPLEX && h->in_dtype == h0->in_dtype && h->out_dtype == h->in_dtype &&
               h->decim == h0->decim && h->ntaps == h0->ntaps && h->bfrag_host == h0->bfrag_host &&
               (ns[c] == 0 || (ins[c] && is_device_ptr(ins[c]))) &&
               (!out_iq[c] || is_device_ptr(out_iq[c])) && (!out_sym[c] || is_device_ptr(out_sym[c]));
        for (size_t e = 0; fuse && e < c; ++e) fuse = hs[e] != h;
    }
    if (!fuse) {
        for (size_t c = 0; c < nch; ++c) {
            const modem_status st = rx_run(hs[c], ins[c], ns[c], false, out_iq[c], out_sym[c], caps[c],
                                           &produced[c], s);
            if (st != MODEM_OK) return st;
        }
        return MODEM_OK;
    }
    for (size_t c = 0; c < nch; ++c) produced[c] = 0;
    std::vector<int64_t> k_first(nch), nout(nch);
    for (size_t c = 0; c < nch; ++c) {
        const modem_rx* h = hs[c];
        rx_range(h->consumed, h->consumed + (int64_t)ns[c], h->decim, h->D, &k_first[c], &nout[c]);
        if ((size_t)nout[c] > caps[c]) return MODEM_ERR_CAPACITY;
    }
    DeviceGuard g(hs[0]->device);
    if (!g.ok) return MODEM_ERR_NO_DEVICE;
    for (size_t c0 = 0; c0 < nch; c0 += mk::kBatchMax) {
        mk::RxBatch b{};
        b.nch = (int32_t)std::min<size_t>(mk::kBatchMax, nch - c0);
        for (int i = 0; i < b.nch; ++i) {
            const size_t c = c0 + (size_t)i;
            rx_fill(hs[c], ins[c], ns[c], out_iq[c], out_sym[c], k_first[c], nout[c], b.p[i]);
        }
        HIP_TRY(mk::launch_rx_mfma_batch(b, (int)hs[0]->decim, hs[0]->mfma_ksteps, hs[0]->d_bfrag,
                                         hs[0]->in_dtype, s));
        for (int i = 0; i < b.nch; ++i) {
            const size_t c = c0 + (size_t)i;
            hs[c]->hcur ^= 1;
            hs[c]->consumed += (int64_t)ns[c];
            produced[c] = (size_t)nout[c];
        }
    }
    return MODEM_OK;
}
uint64_t modem_rx_sample(const modem_rx* h) { return h ? h->c0 + (uint64_t)h->consumed : 0; }
modem_status modem_rx_destroy(modem_rx* h) { delete h; return MODEM_OK; }

// ---------------------------------------------------------------------------- chain ----
// A prepared TX -> RX step over fixed device buffers: the buffers' kinds are checked once here,
// so a step is one launch (modem_chain.hip: TX and RX of the period fused, where the filters
// and the call's geometry allow; MODEM_CHAIN_FUSED=0 in the environment at create time turns
// it off) or the two launches, and the state updates (tx_run / rx_run minus the pointer
// queries and staging decisions, ~1 us of host time each per call).
struct modem_chain {
    bool fused = true;
    int last = -1;             // how the last run ran (modem_chain_fused)
    bool verbose = false;      // MODEM_CHAIN_VERBOSE=1: why a run took the two launches (stderr)
    modem_tx* tx = nullptr;
    modem_rx* rx = nullptr;
    const uint8_t* bits = nullptr;
    size_t nbits = 0;
    void* samples = nullptr;
    size_t cap = 0;
    void* out_iq = nullptr;
    uint8_t* out_sym = nullptr;
    size_t out_cap = 0;
};

modem_status modem_chain_create(modem_tx* tx, modem_rx* rx, const uint8_t* bits, size_t nbits, void* samples,
                                size_t cap, void* out_iq, uint8_t* out_sym, size_t out_cap, modem_chain** out) {
    if (!tx || !rx || !out || !samples || (nbits && !bits)) return MODEM_ERR_INVALID_ARG;
    *out = nullptr;
    if (tx->device != rx->device) return MODEM_ERR_INVALID_ARG;
    // the RX reads what the TX writes: interleaved complex samples of one dtype
    if (tx->out_mode == MODEM_OUT_REAL || rx->in_dtype != tx->dtype) return MODEM_ERR_INVALID_ARG;
    const int dev = tx->device;
    if ((nbits && ptr_kind(bits, dev) != PTR_DEVICE) || ptr_kind(samples, dev) != PTR_DEVICE ||
        (out_iq && ptr_kind(out_iq, dev) != PTR_DEVICE) || (out_sym && ptr_kind(out_sym, dev) != PTR_DEVICE))
        return MODEM_ERR_INVALID_ARG;
    modem_chain* c = new (std::nothrow) modem_chain;
    if (!c) return MODEM_ERR_ALLOC;
    c->tx = tx; c->rx = rx; c->bits = bits; c->nbits = nbits; c->samples = samples; c->cap = cap;
    c->out_iq = out_iq; c->out_sym = out_sym; c->out_cap = out_cap;
    const char* env = std::getenv("MODEM_CHAIN_FUSED");
    c->fused = !(env && env[0] == '0');
    const char* verb = std::getenv("MODEM_CHAIN_VERBOSE");
    c->verbose = verb && verb[0] == '1';
    *out = c;
    return MODEM_OK;
}

modem_status modem_chain_run(modem_chain* c, size_t* produced, size_t* produced_out, void* stream) {
    if (!c || !produced || !produced_out) return MODEM_ERR_INVALID_ARG;
    *produced = *produced_out = 0;
    modem_tx* tx = c->tx;
    modem_rx* rx = c->rx;
    const hipStream_t s = (hipStream_t)stream;
    const uint64_t total = (uint64_t)tx->ncarry + c->nbits;
    const int64_t nsym = (int64_t)(total / tx->bps);
    const int ncarry_new = (int)(total - (uint64_t)nsym * tx->bps);
    const size_t nsamp = (size_t)nsym * tx->sps;
    if (nsamp > c->cap) return MODEM_ERR_CAPACITY;
    int64_t k_first, nout;
    rx_range(rx->consumed, rx->consumed + (int64_t)nsamp, rx->decim, rx->D, &k_first, &nout);
    if ((size_t)nout > c->out_cap) return MODEM_ERR_CAPACITY;
    DeviceGuard g(tx->device);
    if (!g.ok) return MODEM_ERR_NO_DEVICE;
    modem_status st;
    const bool eligible = c->fused && !tx->ph_kind && tx->mfma_ksteps > 0 && rx->mfma_ksteps > 0 &&
                          rx->mix == MODEM_MIX_COMPLEX && tx->out_mode == MODEM_OUT_IQ_MIXED &&
                          rx->out_dtype == rx->in_dtype && tx->sps == rx->decim && nout > 0;
    if (c->verbose && !eligible)
        std::fprintf(stderr, "modem_chain_run: two launches (fused %d ph %d tx ks %d rx ks %d mix %d out_mode %d "
                     "dtypes %d/%d sps %u decim %u nout %lld)\n", (int)c->fused, (int)tx->ph_kind, tx->mfma_ksteps,
                     rx->mfma_ksteps, (int)rx->mix, (int)tx->out_mode, (int)rx->in_dtype, (int)rx->out_dtype,
                     (unsigned)tx->sps, (unsigned)rx->decim, (long long)nout);
    if (eligible) {
        mk::TxParams tp{};
        tx_fill(tx, c->bits, c->nbits, false, c->samples, nsym, ncarry_new, nsamp, tp);
        mk::RxParams rp{};
        rx_fill(rx, c->samples, nsamp, c->out_iq, c->out_sym, k_first, nout, rp);
        int form = 1;
        const hipError_t e = mk::launch_chain_mfma(tp, (int)tx->sps, tx->mfma_ksteps, tx->d_bfrag, rp, rx->mfma_ksteps,
                                                   rx->d_bfrag, tx->dtype, s, &form);
        if (e == hipSuccess) {
            c->last = form;
            tx_advance(tx, false, nsym, ncarry_new, nsamp);
            rx_advance(rx, nsamp);
            *produced = nsamp;
            *produced_out = (size_t)nout;
            return MODEM_OK;
        }
        if (e != hipErrorNotSupported) { (void)hipGetLastError(); return MODEM_ERR_HIP; }
        if (c->verbose) std::fprintf(stderr, "modem_chain_run: no fused form for this call (two launches)\n");
    }
    if ((st = tx_launch(tx, c->bits, c->nbits, false, c->samples, nsym, ncarry_new, nsamp, s))) return st;
    if ((st = rx_launch(rx, c->samples, nsamp, nout ? c->out_iq : nullptr, nout ? c->out_sym : nullptr, k_first,
                        nout, s)))
        return st;
    c->last = 0;
    *produced = nsamp;
    *produced_out = (size_t)nout;
    return MODEM_OK;
}

int modem_chain_fused(const modem_chain* c) { return c ? c->last : -1; }

modem_status modem_chain_destroy(modem_chain* c) { delete c; return MODEM_OK; }

// ----------------------------------------------------------------------- chain batch ----
// A prepared period of a channel bank over fixed device buffers (BASELINE config 4): the
// handles' batch compatibility and the buffers' kinds are checked once here (modem_tx_process_batch
// and modem_rx_process_batch check them on every call: a pointer-attribute query per buffer and a
// comparison of the handles' fragment tables, ~10 us per 4-channel TX call, which held C4's
// channel groups to the host's rate), so a run is the launches and the state updates.
struct modem_chain_batch {
    std::vector<modem_tx*> tx;
    std::vector<modem_rx*> rx;
    std::vector<const uint8_t*> bits;
    std::vector<size_t> nbits, caps, out_caps;
    std::vector<void*> samples, out_iq;
    std::vector<uint8_t*> out_sym;
    size_t group = mk::kBatchMax;
    // Two lanes: group k's TX and RX launches go to the caller's stream (k even) or to the plan's
    // own stream (k odd), joined to the caller's stream by events at the start and the end of a
    // run, so that a group's RX runs beside the next group's TX (each launch's tail of straggling
    // workgroups is filled by the other lane's head). A group stays on its lane from run to run,
    // so each handle's calls keep their order. C4's 64-channel job: 1.049 -> 0.950 ms per step
    // in groups of 8, 1.090 -> 0.948 in groups of 4 (profiles/r05_c4_job.txt).
    // MODEM_CHAIN_BATCH_LANES=1 in the environment at create time: one lane.
    hipStream_t side = nullptr;
    hipEvent_t ev_start = nullptr, ev_end = nullptr;
    bool failed = false;                // a launch of a run failed (modem_chain_batch_run)
    ~modem_chain_batch() {
        if (ev_start) (void)hipEventDestroy(ev_start);
        if (ev_end) (void)hipEventDestroy(ev_end);
        if (side) (void)hipStreamDestroy(side);
    }
};

modem_status modem_chain_batch_create(modem_tx* const* txs, modem_rx* const* rxs, size_t nch, size_t group,
                                      const uint8_t* const* bits, const size_t* nbits, void* const* samples,
                                      const size_t* caps, void* const* out_iq, uint8_t* const* out_sym,
                                      const size_t* out_caps, modem_chain_batch** out) {
    if (!out) return MODEM_ERR_INVALID_ARG;
    *out = nullptr;
    if (!txs || !rxs || nch == 0 || group < 1 || group > (size_t)mk::kBatchMax || !bits || !nbits || !samples ||
        !caps || !out_iq || !out_sym || !out_caps)
        return MODEM_ERR_INVALID_ARG;
    const modem_tx* t0 = txs[0];
    const modem_rx* r0 = rxs[0];
    if (!t0 || !r0) return MODEM_ERR_INVALID_ARG;
    const int dev = t0->device;
    for (size_t c = 0; c < nch; ++c) {
        const modem_tx* t = txs[c];
        const modem_rx* r = rxs[c];
        if (!t || !r || t->device != dev || r->device != dev || !samples[c] || (nbits[c] && !bits[c]))
            return MODEM_ERR_INVALID_ARG;
        for (size_t e = 0; e < c; ++e)
            if (txs[e] == t || rxs[e] == r) return MODEM_ERR_INVALID_ARG;   // a handle at most once
        // the RX reads what the TX writes: interleaved complex samples of one dtype
        if (t->out_mode != MODEM_OUT_IQ_MIXED || r->in_dtype != t->dtype) return MODEM_ERR_INVALID_ARG;
        if ((nbits[c] && ptr_kind(bits[c], dev) != PTR_DEVICE) || ptr_kind(samples[c], dev) != PTR_DEVICE ||
            (out_iq[c] && ptr_kind(out_iq[c], dev) != PTR_DEVICE) ||
            (out_sym[c] && ptr_kind(out_sym[c], dev) != PTR_DEVICE))
            return MODEM_ERR_INVALID_ARG;
        // one matrix-core configuration per side (the batch kernels' conditions)
        if (t->ph_kind != 0 || t->mfma_ksteps <= 0 || t->mfma_ksteps != t0->mfma_ksteps || t->dtype != t0->dtype ||
            t->sps != t0->sps || t->bps != t0->bps || t->ntaps != t0->ntaps || t->q_offset != 0 ||
            t->bfrag_host != t0->bfrag_host)
            return MODEM_ERR_UNSUPPORTED;
        if (r->mfma_ksteps <= 0 || r->mfma_ksteps != r0->mfma_ksteps || r->mix != MODEM_MIX_COMPLEX ||
            r->in_dtype != r0->in_dtype || r->out_dtype != r->in_dtype || r->decim != r0->decim ||
            r->ntaps != r0->ntaps || r->bfrag_host != r0->bfrag_host)
            return MODEM_ERR_UNSUPPORTED;
    }
    modem_chain_batch* b = new (std::nothrow) modem_chain_batch;
    if (!b) return MODEM_ERR_ALLOC;
    const char* lanes = std::getenv("MODEM_CHAIN_BATCH_LANES");
    if (nch > group && !(lanes && lanes[0] == '1')) {
        DeviceGuard g(dev);
        if (!g.ok) { delete b; return MODEM_ERR_NO_DEVICE; }
        if (hipStreamCreateWithFlags(&b->side, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&b->ev_start, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&b->ev_end, hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            delete b;
            return MODEM_ERR_HIP;
        }
    }
    b->tx.assign(txs, txs + nch);
    b->rx.assign(rxs, rxs + nch);
    b->bits.assign(bits, bits + nch);
    b->nbits.assign(nbits, nbits + nch);
    b->samples.assign(samples, samples + nch);
    b->caps.assign(caps, caps + nch);
    b->out_iq.assign(out_iq, out_iq + nch);
    b->out_sym.assign(out_sym, out_sym + nch);
    b->out_caps.assign(out_caps, out_caps + nch);
    b->group = group;
    *out = b;
    return MODEM_OK;
}

// The launches of one run, group by group (after the checks of modem_chain_batch_run).
static modem_status chain_batch_launch(modem_chain_batch* b, hipStream_t s, size_t* produced, size_t* produced_out) {
    const size_t nch = b->tx.size();
    int64_t nsym[mk::kBatchMax], k_first[mk::kBatchMax], nout[mk::kBatchMax];
    int ncarry_new[mk::kBatchMax];
    for (size_t c0 = 0; c0 < nch; c0 += b->group) {
        const int n = (int)std::min(b->group, nch - c0);
        const hipStream_t ls = b->side && (c0 / b->group) % 2 ? b->side : s;   // this group's lane
        mk::TxBatch tb{};
        tb.nch = n;
        uint64_t launch_bytes = 0;
        for (int i = 0; i < n; ++i) {
            const size_t c = c0 + (size_t)i;
            const modem_tx* t = b->tx[c];
            const uint64_t total = (uint64_t)t->ncarry + b->nbits[c];
            nsym[i] = (int64_t)(total / t->bps);
            ncarry_new[i] = (int)(total - (uint64_t)nsym[i] * t->bps);
            const size_t ns = (size_t)nsym[i] * t->sps;
            tx_fill(t, b->bits[c], b->nbits[c], false, b->samples[c], nsym[i], ncarry_new[i], ns, tb.p[i]);
            launch_bytes += (uint64_t)ns * tx_sample_bytes(t);
        }
        for (int i = 0; i < n; ++i)
            tb.p[i].nt_below = tx_nt_below(nsym[i] * (int64_t)b->tx[c0 + i]->sps, launch_bytes, false);
        const modem_tx* t0 = b->tx[c0];
        HIP_TRY(mk::launch_tx_mfma_batch(tb, (int)t0->sps, t0->mfma_ksteps, t0->d_bfrag, t0->dtype, ls));
        mk::RxBatch rb{};
        rb.nch = n;
        for (int i = 0; i < n; ++i) {
            const size_t c = c0 + (size_t)i;
            modem_tx* t = b->tx[c];
            const size_t ns = (size_t)nsym[i] * t->sps;
            tx_advance(t, false, nsym[i], ncarry_new[i], ns);
            modem_rx* r = b->rx[c];
            rx_range(r->consumed, r->consumed + (int64_t)ns, r->decim, r->D, &k_first[i], &nout[i]);
            rx_fill(r, b->samples[c], ns, b->out_iq[c], b->out_sym[c], k_first[i], nout[i], rb.p[i]);
            if (produced) produced[c] = ns;
            if (produced_out) produced_out[c] = (size_t)nout[i];
        }
        const modem_rx* r0 = b->rx[c0];
        HIP_TRY(mk::launch_rx_mfma_batch(rb, (int)r0->decim, r0->mfma_ksteps, r0->d_bfrag, r0->in_dtype, ls));
        for (int i = 0; i < n; ++i) rx_advance(b->rx[c0 + i], (size_t)nsym[i] * b->tx[c0 + i]->sps);
    }
    return MODEM_OK;
}

modem_status modem_chain_batch_run(modem_chain_batch* b, size_t* produced, size_t* produced_out, void* stream) {
    if (!b) return MODEM_ERR_INVALID_ARG;
    // a launch failed in an earlier run: some groups' handles advanced and others not, so the
    // channels' streams no longer line up (the plan and its handles are unusable)
    if (b->failed) return MODEM_ERR_HIP;
    const size_t nch = b->tx.size();
    const hipStream_t s = (hipStream_t)stream;
    // every channel's call sizes first: an error here leaves every handle untouched
    for (size_t c = 0; c < nch; ++c) {
        const modem_tx* t = b->tx[c];
        const uint64_t total = (uint64_t)t->ncarry + b->nbits[c];
        const int64_t ns = (int64_t)(total / t->bps);
        if ((size_t)ns * t->sps > b->caps[c]) return MODEM_ERR_CAPACITY;
        int64_t k0, k;
        rx_range(b->rx[c]->consumed, b->rx[c]->consumed + ns * (int64_t)t->sps, b->rx[c]->decim, b->rx[c]->D, &k0, &k);
        if ((size_t)k > b->out_caps[c]) return MODEM_ERR_CAPACITY;
    }
    DeviceGuard g(b->tx[0]->device);
    if (!g.ok) return MODEM_ERR_NO_DEVICE;
    if (b->side) {                              // the plan's lane starts after what precedes the run
        HIP_TRY(hipEventRecord(b->ev_start, s));
        HIP_TRY(hipStreamWaitEvent(b->side, b->ev_start, 0));
    }
    const modem_status st = chain_batch_launch(b, s, produced, produced_out);
    if (b->side) {                              // the caller's stream continues after both lanes:
        // also after a failed launch (best effort), so that the caller's stream is still ordered
        // after the side lane's kernels already queued
        const bool joined = hipEventRecord(b->ev_end, b->side) == hipSuccess &&
                            hipStreamWaitEvent(s, b->ev_end, 0) == hipSuccess;
        if (st == MODEM_OK && !joined) { (void)hipGetLastError(); b->failed = true; return MODEM_ERR_HIP; }
    }
    if (st != MODEM_OK) b->failed = true;
    return st;
}

modem_status modem_chain_batch_destroy(modem_chain_batch* b) { delete b; return MODEM_OK; }

// ----------------------------------------------------------------------------- FIR ----
struct modem_fir {
    int device = 0;
    uint32_t L = 0;
    float* d_taps = nullptr;
    float* d_hist[2] = {nullptr, nullptr};
    int hcur = 0;
    Stage in_stage, out_stage;
    ~modem_fir() {
        DeviceGuard g(device);
        for (void* p : {(void*)d_taps, (void*)d_hist[0], (void*)d_hist[1]}) if (p) (void)hipFree(p);
    }
};

modem_status modem_fir_create(const float* taps, uint32_t ntaps, int device, modem_fir** out) {
    // FIRFilter::new(&[]) would divide by zero in add() (fir.rs:31): reject it here.
    if (!out || !taps || ntaps < 1 || ntaps > (uint32_t)mk::kMaxTaps) return MODEM_ERR_INVALID_ARG;
    *out = nullptr;
    if (!device_ok(device)) return MODEM_ERR_NO_DEVICE;
    DeviceGuard g(device);
    if (!g.ok) return MODEM_ERR_NO_DEVICE;
    modem_fir* h = new (std::nothrow) modem_fir;
    if (!h) return MODEM_ERR_ALLOC;
    h->device = device;
    h->L = ntaps;
    modem_status st;
    if ((st = dalloc(&h->d_taps, ntaps)) || (st = dalloc(&h->d_hist[0], ntaps)) ||
        (st = dalloc(&h->d_hist[1], ntaps))) { delete h; return st; }
    if (hipMemcpy(h->d_taps, taps, ntaps * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipGetLastError(); delete h; return MODEM_ERR_HIP;
    }
    *out = h;
    return MODEM_OK;
}

modem_status modem_fir_process(modem_fir* h, const float* in, float* out, size_t n, void* stream) {
    if (!h || (n && (!in || !out))) return MODEM_ERR_INVALID_ARG;
    const PtrKind ki = n ? ptr_kind(in, h->device) : PTR_DEVICE, ko = n ? ptr_kind(out, h->device) : PTR_DEVICE;
    if (ki == PTR_FOREIGN || ko == PTR_FOREIGN) return MODEM_ERR_INVALID_ARG;
    DeviceGuard g(h->device);
    if (!g.ok) return MODEM_ERR_NO_DEVICE;
    hipStream_t s = (hipStream_t)stream;
    modem_status st;
    const float* din = in;
    float* dout = out;
    if (ki == PTR_HOST) {
        if ((st = h->in_stage.ensure(n * sizeof(float)))) return st;
        HIP_TRY(hipMemcpyAsync(h->in_stage.p, in, n * sizeof(float), hipMemcpyHostToDevice, s));
        din = static_cast<const float*>(h->in_stage.p);
    }
    const bool host_out = ko == PTR_HOST;
    if (host_out) {
        if ((st = h->out_stage.ensure(n * sizeof(float)))) return st;
        dout = static_cast<float*>(h->out_stage.p);
    }
    mk::FirParams p{};
    p.x = din;
    p.hist = h->d_hist[h->hcur];
    p.hist_new = h->d_hist[h->hcur ^ 1];
    p.y = dout;
    p.taps = h->d_taps;
    p.N = (int64_t)n;
    p.L = (int)h->L;
    HIP_TRY(mk::launch_fir(p, s));
    h->hcur ^= 1;
    if (host_out) HIP_TRY(hipMemcpyAsync(out, dout, n * sizeof(float), hipMemcpyDeviceToHost, s));
    if (host_out || din != in) HIP_TRY(hipStreamSynchronize(s));
    return MODEM_OK;
}

modem_status modem_fir_destroy(modem_fir* h) { delete h; return MODEM_OK; }

modem_status modem_prng_bits(uint64_t seed, uint8_t* out, size_t nbits, int device, void* stream) {
    if (nbits && !out) return MODEM_ERR_INVALID_ARG;
    if (nbits && (!is_device_ptr(out) || foreign_ptr(out, device))) return MODEM_ERR_INVALID_ARG;
    if (!device_ok(device)) return MODEM_ERR_NO_DEVICE;
    DeviceGuard g(device);
    if (!g.ok) return MODEM_ERR_NO_DEVICE;
    HIP_TRY(mk::launch_prng_bits(seed, out, nbits, (hipStream_t)stream));
    return MODEM_OK;
}

}  // extern "C"
