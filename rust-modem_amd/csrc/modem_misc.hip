// rust-modem_amd/csrc/modem_misc.hip — FIRFilter (fir.rs:3-35) as a block kernel, the
// device carrier-phase path (tests) and the splitmix64 bit generator (synthetic input).
#include "modem_device.h"

namespace mk {

// ------------------------------------------------------------------- FIRFilter (real) ----
// y[n] = ((0 + h[0] x[n]) + h[1] x[n-1]) + ... (fir.rs:18-34: FIRFilter::calc folds from the
// newest sample, one f32 multiply and one f32 add per tap, no fusion) — bit-identical to
// FIRFilter::add. 256 lanes x 16 outputs per workgroup.
constexpr int kFirR = 16, kFirNT = 256, kFirTS = kFirR * kFirNT;

__global__ __launch_bounds__(256) void fir_real(const FirParams p) {
#pragma clang fp contract(off)
    extern __shared__ __attribute__((aligned(16))) float flds[];
    const int tid = threadIdx.x, L = p.L;
    if (blockIdx.x == 0)
        for (int i = tid; i < L - 1; i += kFirNT) {
            const int64_t q = p.N - (L - 1) + i;
            p.hist_new[i] = q >= 0 ? p.x[q] : p.hist[q + L - 1];
        }
    const int64_t n0 = (int64_t)blockIdx.x * kFirTS;
    if (n0 >= p.N) return;
    for (int e = tid; e < kFirTS + L - 1; e += kFirNT) {
        const int64_t q = n0 - (L - 1) + e;
        flds[1 + e] = q < 0 ? p.hist[q + L - 1] : (q < p.N ? p.x[q] : 0.f);
    }
    __syncthreads();
    float acc[kFirR];
#pragma unroll
    for (int r = 0; r < kFirR; ++r) acc[r] = 0.f;
    const float* base = flds + 1 + tid * kFirR + (L - 1);
    float win[kFirR];
#pragma unroll
    for (int r = 0; r < kFirR; ++r) win[r] = base[r];
    cfloat* taps = (cfloat*)p.taps;
    int k = 0;
    for (; k + 8 <= L; k += 8) {
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const float h = taps[k + c];
#pragma unroll
            for (int r = 0; r < kFirR; ++r) acc[r] = acc[r] + win[r] * h;
#pragma unroll
            for (int r = kFirR - 1; r > 0; --r) win[r] = win[r - 1];
            win[0] = base[-(k + c + 1)];
        }
    }
    for (; k < L; ++k) {
        const float h = taps[k];
#pragma unroll
        for (int r = 0; r < kFirR; ++r) acc[r] = acc[r] + win[r] * h;
#pragma unroll
        for (int r = kFirR - 1; r > 0; --r) win[r] = win[r - 1];
        win[0] = base[-(k + 1)];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kFirR; ++r) flds[tid * kFirR + r] = acc[r];
    __syncthreads();
    const int64_t nh = p.N - n0 < kFirTS ? p.N - n0 : kFirTS;
    for (int i = tid; i < nh; i += kFirNT) p.y[n0 + i] = flds[i];
}

// ----------------------------------------------------------- carrier phases (tests) ----
__global__ __launch_bounds__(256) void carrier_phases(float w, uint64_t s0, size_t n, int exact_idx,
                                                      float* out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = carrier_phase(w, s0 + i, exact_idx != 0);
}

hipError_t launch_phases(float w, uint64_t s0, size_t n, float* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const int exact_idx = (s0 + n) <= (1ull << 53) ? 1 : 0;
    hipLaunchKernelGGL(carrier_phases, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, w, s0, n,
                       exact_idx, out);
    return hipGetLastError();
}

// ------------------------------------------------------------------- splitmix64 bits ----
__global__ __launch_bounds__(256) void prng_bits(uint64_t seed, uint8_t* out, size_t nbits) {
    const size_t w = (size_t)blockIdx.x * blockDim.x + threadIdx.x;   // one 64-bit word
    if (w * 64 >= nbits) return;
    uint64_t z = seed + (uint64_t)(w + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z = z ^ (z >> 31);
    const size_t b0 = w * 64;
    if (b0 + 64 <= nbits && (reinterpret_cast<uintptr_t>(out + b0) & 15) == 0) {
        uint4* o = reinterpret_cast<uint4*>(out + b0);
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            uint32_t wd[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int bit = v * 16 + k * 4;
                wd[k] = (uint32_t)((z >> bit) & 1) | (uint32_t)((z >> (bit + 1)) & 1) << 8 |
                        (uint32_t)((z >> (bit + 2)) & 1) << 16 | (uint32_t)((z >> (bit + 3)) & 1) << 24;
            }
            o[v] = make_uint4(wd[0], wd[1], wd[2], wd[3]);
        }
    } else {
        for (size_t i = b0; i < nbits; ++i) out[i] = (uint8_t)((z >> (i - b0)) & 1);
    }
}


hipError_t launch_fir(const FirParams& p, hipStream_t s) {
    const int64_t nblk = (p.N + kFirTS - 1) / kFirTS;
    const size_t lds = (size_t)(kFirTS + p.L + 1) * sizeof(float);
    hipLaunchKernelGGL(fir_real, dim3((unsigned)(nblk > 0 ? nblk : 1)), dim3(kFirNT), lds, s, p);
    return hipGetLastError();
}

hipError_t launch_prng_bits(uint64_t seed, uint8_t* out, size_t nbits, hipStream_t s) {
    const size_t words = (nbits + 63) / 64;
    const size_t nblk = (words + 255) / 256;
    if (nblk == 0) return hipSuccess;
    hipLaunchKernelGGL(prng_bits, dim3((unsigned)nblk), dim3(256), 0, s, seed, out, nbits);
    return hipGetLastError();
}


}  // namespace mk
