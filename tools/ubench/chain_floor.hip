// The chains' byte patterns with no compute: the measured practical floor of each bench config
// (VERDICT r03 item 1 for C3; r04 "missing" item 2 for the out-of-cache configs). Per period:
// bits in (bps / sps B per sample), samples written (S B) and re-read, decimated I/Q (S / sps)
// + decisions (1 / sps) written, over the product kernels' tiles of 1024 kept instants
// (TS = 1024 sps samples), 256 threads per tile, 16-B accesses.
//
//   c2   QPSK sps 4, f32, 2^20 samples over the small tiles (256 instants, one per workgroup at
//        4 per CU), with the empty persistent launch of that grid (the call's launch floor)
//   c3   16-QAM sps 4, f32, 2^24 samples (19.25 B/sample, 323 MB): the round-4 variants (fused
//        TX/RX tiles in one persistent launch, lag G or 0, write-through stores) besides the two
//        launches
//   c4   8 QPSK channels x 2^22 (one batch launch pair, 2^25 samples, 18.75 B/sample);
//   c4g4 4 channels per launch pair (2^24 samples)
//   c5   256-QAM sps 8, f32, 2^26 samples (18.125 B/sample, 1.22 GB)
//   c5h  the same with f16 samples (9.625 B/sample, 646 MB)
// Every config: the two launches with default-policy TX stores, with non-temporal TX stores,
// with the first half non-temporal (the product's C5 f16 policy), TX alone, RX alone; the RX
// walks its tiles top-down in rounds of the grid, as rx_mfma does.
//
// hipcc -O3 --offload-arch=gfx950 chain_floor.hip -o chain_floor && ./chain_floor [config|all] [pmc]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef unsigned u4v __attribute__((ext_vector_type(4)));

// One config's tile shape. TS samples per tile, S bytes per sample, BB bits bytes per tile,
// IQB I/Q bytes and SYB decision bytes per tile (all multiples of 16 x 256 or of 4 x 256).
template <int TS_, int S_, int BB_, int SPS_>
struct Shape {
    static constexpr int TS = TS_, S = S_, BB = BB_, SPS = SPS_;
    static constexpr int YV = TS * S / 16 / 256;        // 16-B sample vectors per thread
    static constexpr int BV = (BB / 16 + 255) / 256;    // 16-B bit vectors per thread (partial)
    static constexpr int IQB = TS / SPS * S;            // I/Q bytes per tile
    static constexpr int IQV = (IQB / 16 + 255) / 256;  // 16-B I/Q vectors per thread (partial)
    static constexpr int SYB = TS / SPS;                // decision bytes per tile
    static constexpr int SYW = (SYB / 4 + 255) / 256;   // 4-B decision words per thread (partial)
    static_assert(YV >= 1 && TS * S % (16 * 256) == 0 && IQB % 16 == 0 && SYB % 4 == 0, "tile shape");
};

// TX tile t: bits in, samples out (nt: non-temporal stores, as tx_nt_below)
template <class C>
__device__ __forceinline__ void tx_tile(const uint4* __restrict__ bits, uint4* __restrict__ y, int64_t t, bool nt) {
    unsigned v = 0;
#pragma unroll
    for (int k = 0; k < C::BV; ++k) {
        const int i = k * 256 + threadIdx.x;
        if (i * 16 < C::BB) {
            const uint4 b = bits[t * (C::BB / 16) + i];
            v ^= b.x ^ b.y ^ b.z ^ b.w;
        }
    }
    uint4* o = y + t * (C::TS * C::S / 16);
#pragma unroll
    for (int j = 0; j < C::YV; ++j) {
        const u4v w = {v, v + j, v ^ 5u, v - j};
        if (nt) __builtin_nontemporal_store(w, reinterpret_cast<u4v*>(o + j * 256 + threadIdx.x));
        else *reinterpret_cast<u4v*>(o + j * 256 + threadIdx.x) = w;
    }
}
// RX tile t: samples in, I/Q and decisions out
template <class C>
__device__ __forceinline__ void rx_tile(const uint4* __restrict__ y, uint4* __restrict__ iq, unsigned* __restrict__ sym,
                                        int64_t t) {
    const uint4* x = y + t * (C::TS * C::S / 16);
    uint4 a = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < C::YV; ++j) {
        const uint4 v = x[j * 256 + threadIdx.x];
        a.x += v.x; a.y ^= v.y; a.z += v.z; a.w ^= v.w;
    }
    uint4* o = iq + t * (C::IQB / 16);
#pragma unroll
    for (int j = 0; j < C::IQV; ++j)
        if ((j * 256 + (int)threadIdx.x) * 16 < C::IQB) o[j * 256 + threadIdx.x] = make_uint4(a.x + j, a.y, a.z, a.w);
#pragma unroll
    for (int j = 0; j < C::SYW; ++j)
        if ((j * 256 + (int)threadIdx.x) * 4 < C::SYB) sym[t * (C::SYB / 4) + j * 256 + threadIdx.x] = (a.x ^ a.z) & 0x0f0f0f0f;
}

// nt_below: tiles < nt_below store non-temporally
template <class C>
__global__ __launch_bounds__(256) void k_tx(const uint4* bits, uint4* y, int64_t nt, int64_t nt_below) {
    for (int64_t t = blockIdx.x; t < nt; t += gridDim.x) tx_tile<C>(bits, y, t, t < nt_below);
}
template <class C>
__global__ __launch_bounds__(256) void k_rx(const uint4* y, uint4* iq, unsigned* sym, int64_t nt) {
    const int64_t G = gridDim.x, R = (nt + G - 1) / G;      // top-down rounds, as rx_mfma
    for (int64_t r = 0; r < R; ++r) {
        const int64_t t = nt - (r + 1) * G + blockIdx.x;
        if (t >= 0) rx_tile<C>(y, iq, sym, t);
    }
}
// C3 only (round 4): one persistent launch, TX tile t then RX tile t - G (lag G) or t (lag 0)
template <class C>
__global__ __launch_bounds__(256) void k_fused(const uint4* bits, uint4* y, uint4* iq, unsigned* sym, int64_t nt) {
    const int64_t G = gridDim.x;
    int64_t t = blockIdx.x;
    for (; t < nt; t += G) {
        tx_tile<C>(bits, y, t, false);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t - G >= 0) rx_tile<C>(y, iq, sym, t - G);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t - G >= 0 && t - G < nt) rx_tile<C>(y, iq, sym, t - G);   // (a grid larger than the tiles: none)
}
template <class C>
__global__ __launch_bounds__(256) void k_fused0(const uint4* bits, uint4* y, uint4* iq, unsigned* sym, int64_t nt) {
    for (int64_t t = blockIdx.x; t < nt; t += gridDim.x) {
        tx_tile<C>(bits, y, t, false);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        rx_tile<C>(y, iq, sym, t);
    }
}

// an empty persistent grid: the launch floor of a one-tile-per-workgroup call (C2)
__global__ __launch_bounds__(256) void k_empty(unsigned* o) {
    if (o && threadIdx.x == 1023) o[blockIdx.x] = 0;
}

static bool g_quick = false;                     // "pmc": 3 launches each, untimed
template <typename F> static void run(const char* name, double bytes, F f) {
    if (g_quick) { for (int i = 0; i < 3; ++i) f(); (void)hipDeviceSynchronize(); printf("%s\n", name); return; }
    for (int i = 0; i < 100; ++i) f();           // settle the clocks
    (void)hipDeviceSynchronize();
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    float best = 1e30f, sum = 0;
    const int R = 5, K = 100;
    for (int r = 0; r < R; ++r) {
        (void)hipEventRecord(a);
        for (int k = 0; k < K; ++k) f();
        (void)hipEventRecord(b); (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b); ms /= K;
        best = ms < best ? ms : best; sum += ms;
    }
    printf("%-50s min %8.2f us  mean %8.2f us  %6.2f TB/s (min)\n", name, best * 1e3, sum / R * 1e3,
           bytes / (best * 1e-3) / 1e12);
    fflush(stdout);
}

template <class C>
static void config(const char* cname, int64_t nsamp, bool c3_extra, int ncu) {
    const int64_t nt = nsamp / C::TS;
    const size_t bb = (size_t)nt * C::BB, yb = (size_t)nsamp * C::S, iqb = (size_t)nsamp / C::SPS * C::S,
                 syb = (size_t)nsamp / C::SPS;
    uint4 *bits, *y, *iq; unsigned* sym;
    if (hipMalloc(&bits, bb) || hipMalloc(&y, yb) || hipMalloc(&iq, iqb) || hipMalloc(&sym, syb)) {
        printf("%s: hipMalloc failed\n", cname);
        exit(1);
    }
    (void)hipMemset(bits, 1, bb);
    (void)hipMemset(y, 0, yb);
    const double btx = (double)bb + yb, brx = (double)yb + iqb + syb, bch = btx + brx;
    printf("\n[%s] %lld samples, %lld tiles of %d; chain bytes per period %.1f MB (%.4g B/sample)\n", cname,
           (long long)nsamp, (long long)nt, C::TS, bch / 1e6, bch / nsamp);
    for (int per : {2, 4, 8}) {
        const int G = ncu * per;
        char n[112];
        auto two = [&](int64_t ntb) {
            hipLaunchKernelGGL(k_tx<C>, G, 256, 0, 0, bits, y, nt, ntb);
            hipLaunchKernelGGL(k_rx<C>, G, 256, 0, 0, y, iq, sym, nt);
        };
        snprintf(n, sizeof n, "%s two launches grid %d", cname, G);
        run(n, bch, [&] { two(0); });
        snprintf(n, sizeof n, "%s two launches, tx nt stores grid %d", cname, G);
        run(n, bch, [&] { two(nt); });
        snprintf(n, sizeof n, "%s two launches, tx first half nt grid %d", cname, G);
        run(n, bch, [&] { two(nt / 2); });
        if (c3_extra) {
            snprintf(n, sizeof n, "%s fused (tx t, rx t-G) grid %d", cname, G);
            run(n, bch, [&] { hipLaunchKernelGGL(k_fused<C>, G, 256, 0, 0, bits, y, iq, sym, nt); });
            snprintf(n, sizeof n, "%s fused lag 0 (tx t, rx t) grid %d", cname, G);
            run(n, bch, [&] { hipLaunchKernelGGL(k_fused0<C>, G, 256, 0, 0, bits, y, iq, sym, nt); });
        }
        if (per == 4 && nt <= G) {
            snprintf(n, sizeof n, "%s empty launch grid %d", cname, G);
            run(n, 0, [&] { hipLaunchKernelGGL(k_empty, G, 256, 0, 0, (unsigned*)nullptr); });
        }
        snprintf(n, sizeof n, "%s tx alone grid %d", cname, G);
        run(n, btx, [&] { hipLaunchKernelGGL(k_tx<C>, G, 256, 0, 0, bits, y, nt, (int64_t)0); });
        snprintf(n, sizeof n, "%s tx alone, nt stores grid %d", cname, G);
        run(n, btx, [&] { hipLaunchKernelGGL(k_tx<C>, G, 256, 0, 0, bits, y, nt, nt); });
        snprintf(n, sizeof n, "%s rx alone grid %d", cname, G);
        run(n, brx, [&] { hipLaunchKernelGGL(k_rx<C>, G, 256, 0, 0, y, iq, sym, nt); });
    }
    (void)hipFree(bits); (void)hipFree(y); (void)hipFree(iq); (void)hipFree(sym);
}

int main(int argc, char** argv) {
    const char* which = argc > 1 ? argv[1] : "all";
    g_quick = argc > 2 && argv[2][0] == 'p';
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    printf("CUs %d\n", ncu);
    auto on = [&](const char* c) { return !strcmp(which, "all") || !strcmp(which, c); };
    // Shape<samples per tile, bytes per sample, bits bytes per tile, sps>
    if (on("c2")) config<Shape<1024, 8, 512, 4>>("c2", 1 << 20, true, ncu);
    if (on("c3")) config<Shape<4096, 8, 4096, 4>>("c3", 1 << 24, true, ncu);
    if (on("c4")) config<Shape<4096, 8, 2048, 4>>("c4", 1 << 25, false, ncu);
    if (on("c4g4")) config<Shape<4096, 8, 2048, 4>>("c4g4", 1 << 24, false, ncu);
    if (on("c5")) config<Shape<8192, 8, 8192, 8>>("c5", 1 << 26, false, ncu);
    if (on("c5h")) config<Shape<8192, 4, 8192, 8>>("c5h", 1 << 26, false, ncu);
    return 0;
}
