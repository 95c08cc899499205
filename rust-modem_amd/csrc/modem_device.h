// rust-modem_amd/csrc/modem_device.h — device helpers shared by the gfx950 kernel files
// (modem_tx.hip, modem_rx.hip, modem_misc.hip): the bit-exact carrier phase, sin/cos, vector
// helpers, sample I/O and the persistent-grid sizing used by every launcher.
#pragma once
#include "modem_internal.h"

#include <hip/hip_fp16.h>

#include <cstdlib>
#include <map>
#include <mutex>
#include <utility>

namespace mk {

// ----------------------------------------------------------------------------------------
// Bit-exact reference carrier phase: mod_trig(w * (n as f32)).
//   x = fl(w * fl(n)); phase = fl(x - fl(TWO_PI * floor(fl(x / TWO_PI)))).
// fl(x / TWO_PI) is replaced by q1 = q0 + r*RC (q0 = x*RC, r = fma(-q0, TWO_PI, x)):
// q1 differs from the IEEE quotient for some x but floor(q1) == floor(fl(x/TWO_PI)) for
// every non-negative finite f32 (checked exhaustively on the host: tests/test_phase_math.py),
// so the phase is bit-identical. contract(off) keeps TWO_PI*f and the subtraction
// separately rounded, as rustc does.
constexpr float kTwoPi = 0x1.921fb6p+2f;   // std::f32::consts::PI * 2.0 (0x40c90fdb)
constexpr float kRcp2Pi = 0x1.45f306p-3f;  // fl(1 / kTwoPi)

__device__ __forceinline__ float phase_from_f(float w, float nf) {
#pragma clang fp contract(off)
    const float x = w * nf;
    const float q0 = x * kRcp2Pi;
    const float r = __builtin_fmaf(-q0, kTwoPi, x);
    const float q1 = __builtin_fmaf(r, kRcp2Pi, q0);
    const float f = __builtin_floorf(q1);
    const float p = kTwoPi * f;
    return x - p;
}

// (re, im) pair: one v_pk_fma_f32 per complex x real MAC, tap broadcast from an SGPR.
typedef float cf2 __attribute__((ext_vector_type(2)));

// phase_from_f for two indices at once on the packed f32 VALU (v_pk_mul/v_pk_fma/v_pk_add_f32
// round each half exactly as the scalar ops do, so both phases are bit-identical to
// phase_from_f; two samples per issue, floor stays scalar).
__device__ __forceinline__ cf2 phase_from_f2(float w, cf2 nf) {
#pragma clang fp contract(off)
    const cf2 x = nf * w;
    const cf2 q0 = x * kRcp2Pi;
    const cf2 r = __builtin_elementwise_fma(-q0, (cf2){kTwoPi, kTwoPi}, x);
    const cf2 q1 = __builtin_elementwise_fma(r, (cf2){kRcp2Pi, kRcp2Pi}, q0);
    const cf2 f = (cf2){__builtin_floorf(q1.x), __builtin_floorf(q1.y)};
    const cf2 p = f * kTwoPi;
    return x - p;
}

// The same for four indices: two independent packed pairs per step, so that no packed op reads
// the result of the one right before it (gfx950 pads such a read with an s_nop).
typedef float cf4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ cf4 phase_from_f4(float w, cf4 nf) {
#pragma clang fp contract(off)
    // -TWO_PI kept opaque: x + fl(f * -TWO_PI) == fl(x - fl(TWO_PI * f)) (negation is exact), and
    // stays a packed add instead of being folded back into two scalar subtractions
    float ntp = -kTwoPi;
    asm("" : "+s"(ntp));
    const cf4 x = nf * w;
    const cf4 q0 = x * kRcp2Pi;
    const cf4 r = __builtin_elementwise_fma(q0, (cf4){ntp, ntp, ntp, ntp}, x);
    const cf4 q1 = __builtin_elementwise_fma(r, (cf4){kRcp2Pi, kRcp2Pi, kRcp2Pi, kRcp2Pi}, q0);
    const cf4 f = (cf4){__builtin_floorf(q1.x), __builtin_floorf(q1.y), __builtin_floorf(q1.z), __builtin_floorf(q1.w)};
    return x + f * ntp;
}

// `n as f32` with round-to-nearest-even. Below 2^53 (`exact_idx`, checked on the host per
// call) the index is exact as an f64 and one v_cvt_f32_f64 rounds it once, as rustc's u64 -> f32
// does; the hot loops keep a per-lane f64 index and add the per-sample offset in f64 (no
// 32-bit index wrap at 2^32, so streams longer than 4.3 Gsamples stay on the fast paths).
// At and above 2^53 the compiler's exact u64 -> f32 sequence.
__device__ __forceinline__ float idx_f32(double nd) { return (float)nd; }

__device__ __forceinline__ float carrier_phase(float w, uint64_t n, bool exact_idx) {
    const float nf = exact_idx ? idx_f32((double)n) : (float)n;
    return phase_from_f(w, nf);
}

// Same, for n = base + off with a wave-uniform 64-bit base and a 32-bit lane offset. The add is
// done in u64 first: callers may pass a base "before the stream" (wrapped below 0) with an
// offset that brings n back to >= 0, which an f64 add of the two parts would not reproduce.
__device__ __forceinline__ float carrier_phase_off(float w, uint64_t base, int off, bool exact_idx) {
    const uint64_t n = base + (uint64_t)(int64_t)off;
    const float nf = exact_idx ? idx_f32((double)n) : (float)n;
    return phase_from_f(w, nf);
}

// sin/cos of a phase in [0, 2pi] on the hardware v_sin_f32/v_cos_f32 (input in revolutions);
// the sample tolerance is set in tests/test_gpu_parity.py. (The bit-exact libm results of the
// reference's own demodulator: libm_sincosf.h.)
__device__ __forceinline__ void sincos_phase(float ph, float& s, float& c) {
    s = __sinf(ph);
    c = __cosf(ph);
}

// Hardware sin/cos of two phases (what __sinf/__cosf compile to: v_sin/v_cos of phase/2pi,
// here with one packed multiply for both samples).
__device__ __forceinline__ void sincos_phase2(cf2 ph, cf2& s, cf2& c) {
    const cf2 rev = ph * kRcp2Pi;
    s = (cf2){__builtin_amdgcn_sinf(rev.x), __builtin_amdgcn_sinf(rev.y)};
    c = (cf2){__builtin_amdgcn_cosf(rev.x), __builtin_amdgcn_cosf(rev.y)};
}

typedef const __attribute__((address_space(4))) float cfloat;   // wave-uniform -> s_load
__device__ __forceinline__ cf2 ldc(const float2* p) { return *reinterpret_cast<const cf2*>(p); }
__device__ __forceinline__ cf2 cmac(cf2 x, float h, cf2 acc) {
    return __builtin_elementwise_fma(x, (cf2){h, h}, acc);
}


// Output buffers are device (global) memory: every sample store goes through an address-space-1
// view of the caller's pointer, so that it compiles to global_store (counted in vmcnt only). A
// store through a generic pointer is a flat_store, which also counts in lgkmcnt: the compiler then
// cannot wait for an LDS read alone while one is in flight, and every LDS wait after a sample store
// became `s_waitcnt vmcnt(0) lgkmcnt(0)` -- the TX filter's first MFMA of each 16x16 sub-tile waited
// for all the wave's earlier sample stores to complete (profiles/r05_tx_global_stores.txt).
template <typename T> using gptr = __attribute__((address_space(1))) T*;
template <typename T> __device__ __forceinline__ gptr<T> gcast(void* p) { return (gptr<T>)p; }
typedef float gv2f __attribute__((ext_vector_type(2)));     // (HIP's float2 / float4 classes cannot be
typedef float gv4f __attribute__((ext_vector_type(4)));     // assigned through an address-space-1 pointer)
typedef uint32_t gv2u __attribute__((ext_vector_type(2)));

// Buffer descriptor over `bytes` bytes at `base` (wave-uniform inputs made provably uniform).
// Accesses past `bytes` load zeros / are dropped without touching memory.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint32_t bytes) {
    const uint64_t a = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0,
                                             __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// Cache policy of a buffer store (its aux immediate on gfx950): 0 default, 2 non-temporal.
enum { BUF_DEFAULT = 0, BUF_NT = 2 };

template <typename OutT> struct OutIO;
template <> struct OutIO<float> {
    __device__ static void store_pair(void* out, int64_t j, float a, float b, float c, float d) {
        *gcast<gv4f>(reinterpret_cast<float*>(out) + 2 * j) = (gv4f){a, b, c, d};
    }
    __device__ static void store_one(void* out, int64_t j, float a, float b) {
        *gcast<gv2f>(reinterpret_cast<float*>(out) + 2 * j) = (gv2f){a, b};
    }
    __device__ static void store_one_nt(void* out, int64_t j, float a, float b) {   // non-temporal
        __builtin_nontemporal_store((gv2f){a, b}, gcast<gv2f>(reinterpret_cast<float*>(out) + 2 * j));
    }
    __device__ static void store_real_pair(void* out, int64_t j, float a, float b) {
        *gcast<gv2f>(reinterpret_cast<float*>(out) + j) = (gv2f){a, b};
    }
    __device__ static void store_real_one(void* out, int64_t j, float a) {
        *gcast<float>(reinterpret_cast<float*>(out) + j) = a;
    }
};
template <> struct OutIO<__half> {
    __device__ static void store_pair(void* out, int64_t j, float a, float b, float c, float d) {
        const __half2 h0 = __floats2half2_rn(a, b), h1 = __floats2half2_rn(c, d);
        *gcast<gv2u>(reinterpret_cast<__half*>(out) + 2 * j) =
            (gv2u){*reinterpret_cast<const uint32_t*>(&h0), *reinterpret_cast<const uint32_t*>(&h1)};
    }
    __device__ static void store_one(void* out, int64_t j, float a, float b) {
        const __half2 h = __floats2half2_rn(a, b);
        *gcast<uint32_t>(reinterpret_cast<__half*>(out) + 2 * j) = *reinterpret_cast<const uint32_t*>(&h);
    }
    __device__ static void store_one_nt(void* out, int64_t j, float a, float b) {   // non-temporal
        const __half2 h = __floats2half2_rn(a, b);
        __builtin_nontemporal_store(*reinterpret_cast<const uint32_t*>(&h),
                                    gcast<uint32_t>(reinterpret_cast<__half*>(out) + 2 * j));
    }
    __device__ static void store_real_pair(void* out, int64_t j, float a, float b) {
        const __half2 h = __floats2half2_rn(a, b);
        *gcast<uint32_t>(reinterpret_cast<__half*>(out) + j) = *reinterpret_cast<const uint32_t*>(&h);
    }
    __device__ static void store_real_one(void* out, int64_t j, float a) {
        const __half h = __float2half_rn(a);
        *gcast<uint16_t>(reinterpret_cast<__half*>(out) + j) = *reinterpret_cast<const uint16_t*>(&h);
    }
};

enum { OUT_IQ_MIXED = 0, OUT_IQ_BASEBAND = 1, OUT_REAL = 2 };


// Sliding register window: win[0] <- v, the rest shift up.
template <int R>
__device__ __forceinline__ void shift_in(cf2 (&win)[R], cf2 v) {
#pragma unroll
    for (int r = R - 1; r > 0; --r) win[r] = win[r - 1];
    win[0] = v;
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Keep a loaded value in its register: an opaque asm use stops the compiler from
// rematerialising the load inside a tile loop (where its vmcnt wait would also drain the
// next tile's prefetch, since vector-memory counters retire in issue order).
__device__ __forceinline__ void pin(float& v) { asm volatile("" : "+v"(v)); }

// ---------------------------------------------------------------------- dispatch ----
// Persistent grids: resident workgroups per CU (occupancy API, cached per kernel and LDS
// size) x CUs, never more than the number of tiles.
static inline int device_cus() {
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (cus[dev] == 0) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cus[dev] = n;
    }
    return cus[dev];
}

static std::mutex g_occ_mu;
static std::map<std::pair<const void*, size_t>, int> g_occ;

static inline int resident_blocks(const void* kernel, int threads, size_t lds) {
    std::lock_guard<std::mutex> lk(g_occ_mu);
    auto key = std::make_pair(kernel, lds);
    auto it = g_occ.find(key);
    if (it != g_occ.end()) return it->second;
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, threads, lds) != hipSuccess || occ <= 0) {
        (void)hipGetLastError();
        occ = 1;
    }
    g_occ[key] = occ;
    return occ;
}


static inline unsigned persistent_grid(const void* kernel, int threads, size_t lds, int64_t ntiles,
                                       int cap_per_cu = 0) {
    int per_cu = resident_blocks(kernel, threads, lds);
    if (cap_per_cu > 0 && cap_per_cu < per_cu) per_cu = cap_per_cu;
    const int64_t cap = (int64_t)per_cu * device_cus();
    const int64_t g = ntiles < cap ? ntiles : cap;
    return (unsigned)(g > 0 ? g : 1);
}


// XCD-chunked tile slots of a persistent grid (tx_mfma / rx_mfma): workgroups are dealt to the 8
// XCDs round-robin (block b on XCD b mod 8), and a grid-strided walk (tile slot + k nb) puts
// neighbouring tiles on different XCDs, so a tile's window halo (the bits before a TX tile, the
// samples before an RX tile) is read from another XCD's L2 or from HBM. Block 8 j + x takes slot
// (8 (j / c) + x) c + j mod c instead: runs of c consecutive tiles per XCD, the slot still a
// bijection on [0, nb) when 8 c divides nb (xcd_chunk), every XCD's tiles advancing by nb per
// round, and tile i on XCD (i / c) mod 8 for any such grid, so the TX and the RX still meet on
// the XCD that wrote a tile. c = 1 is the plain walk.
__device__ __forceinline__ int64_t xcd_slot(int64_t bid, int c) {
    if (c <= 1) return bid;
    const int64_t j = bid >> 3, x = bid & 7;
    return ((j / c) * 8 + x) * c + j % c;
}
// the chunk for a grid of nb workgroups: MODEM_XCD_CHUNK (default 8) halved until 8 c divides nb
static inline int xcd_chunk(int64_t nb) {
    static const int c0 = [] {
        const char* e = std::getenv("MODEM_XCD_CHUNK");
        const int v = e ? std::atoi(e) : 8;
        return v >= 1 ? v : 1;
    }();
    int c = c0;
    while (c > 1 && nb % (8 * (int64_t)c) != 0) c >>= 1;
    return c;
}


// acc_re/acc_im += sum_s A_s * B_s over NKS k-steps; A_s (complex) is read from LDS at
// arow[off(s)], PD k-steps ahead of its MFMA pair (explicit software pipeline: the
// scheduling barriers keep the compiler from collapsing it to one read of look-ahead).
template <int NKS, int PD, typename OffF>
__device__ __forceinline__ void mfma_chain(const float2* arow, OffF off, const float (&bf)[NKS],
                                           f32x4& dre, f32x4& dim) {
    float2 a[PD];
#pragma unroll
    for (int s = 0; s < PD && s < NKS; ++s) a[s] = arow[off(s)];
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
        const float2 cur = a[s % PD];
        if (s + PD < NKS) a[s % PD] = arow[off(s + PD)];
        dre = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.x, bf[s], dre, 0, 0, 0);
        dim = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.y, bf[s], dim, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// The same chain with B also read from LDS, at brow[4*s] (a Toeplitz band table: one
// conflict-free ds_read_b32 per k-step instead of NKS fragment registers per lane).
template <int NKS, int PD, typename OffF>
__device__ __forceinline__ void mfma_chain_lb(const float2* arow, OffF off, const float* brow,
                                              f32x4& dre, f32x4& dim) {
    float2 a[PD];
    float b[PD];
#pragma unroll
    for (int s = 0; s < PD && s < NKS; ++s) {
        a[s] = arow[off(s)];
        b[s] = brow[4 * s];
    }
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
        const float2 cur = a[s % PD];
        const float cb = b[s % PD];
        if (s + PD < NKS) {
            a[s % PD] = arow[off(s + PD)];
            b[s % PD] = brow[4 * (s + PD)];
        }
        dre = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.x, cb, dre, 0, 0, 0);
        dim = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.y, cb, dim, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// The fused small call's LDS sample window (RawOut / RxHandoff): element i lives at raw_pos(i).
// raw_pos swaps 8-B elements inside aligned groups of 4 by bits 5-6 of the index. The RX reads
// its staging quads there (lane l: elements 4 l + j): unswizzled, lanes l and l + 8 hit the same
// bank pair of a ds_read_b64 (bank = element mod 32), a 4-way conflict on every read (C2's
// chain_small: ~100 conflict cycles per workgroup, 102,400 per launch); swizzled, the 32 lanes of
// each group cover 32 distinct elements mod 32 for any start. The TX's 16 consecutive lanes per
// ds_write_b64 group write 16 consecutive elements of a 16-aligned run: still distinct mod 16.
__device__ __forceinline__ int64_t raw_pos(int64_t i) { return i ^ ((i >> 5) & 3); }

}  // namespace mk
