// The C3 chain's byte pattern with no compute (the measured practical floor).
// Per 2^24-sample period: bits in 16 MiB (1 B/sample), samples written 128 MiB, the same samples
// re-read 128 MiB, decimated I/Q 32 MiB + decisions 4 MiB written (19.25 B/sample, 323 MB).
//
//   two   : the two launches of the product chain, as streaming kernels over 4096-sample tiles
//           (tile = the TX/RX kernels' tile: 1024 symbols / 1024 instants at sps 4); the RX
//           pattern walks tiles top-down as rx_mfma does.
//   fused : ONE persistent launch, each workgroup alternating TX tile t and RX tile t - G (the
//           tile it wrote one round earlier; G = the grid), the re-read still through global
//           loads of the sample buffer.
//   tx / rx alone, and a plain write-then-read of 128 MiB for reference.
//
// hipcc -O3 --offload-arch=gfx950 chain_floor.hip -o chain_floor && ./chain_floor
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define NS (1 << 24)                 // samples per period
#define TS 4096                      // samples per tile
#define NT (NS / TS)                 // tiles

// TX tile: 4096 bits bytes in (16 B per thread), 32 KiB of samples out (8 float4 per thread).
__device__ __forceinline__ void tx_tile(const uint4* __restrict__ bits, float4* __restrict__ y, int t) {
    const uint4 b = bits[(size_t)t * 256 + threadIdx.x];
    const float v = (float)(b.x ^ b.y ^ b.z ^ b.w);
    float4* o = y + (size_t)t * (TS * 8 / 16);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j * 256 + threadIdx.x] = make_float4(v, v + j, v, v - j);
}
// RX tile: 32 KiB of samples in (8 float4 per thread), 8 KiB of I/Q (2 float4 per thread) and
// 1 KiB of decisions (4 B per thread) out.
__device__ __forceinline__ void rx_tile(const float4* __restrict__ y, float4* __restrict__ iq,
                                        unsigned* __restrict__ sym, int t) {
    const float4* x = y + (size_t)t * (TS * 8 / 16);
    float4 a = make_float4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float4 v = x[j * 256 + threadIdx.x];
        a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    float4* o = iq + (size_t)t * 512;
    o[threadIdx.x] = a;
    o[256 + threadIdx.x] = make_float4(a.w, a.z, a.y, a.x);
    sym[(size_t)t * 256 + threadIdx.x] = __float_as_uint(a.x) & 0x0f0f0f0f;
}

__global__ __launch_bounds__(256) void k_tx(const uint4* bits, float4* y) {
    for (int t = blockIdx.x; t < NT; t += gridDim.x) tx_tile(bits, y, t);
}
__global__ __launch_bounds__(256) void k_rx(const float4* y, float4* iq, unsigned* sym) {
    // top-down rounds, as rx_mfma walks C3
    const int G = gridDim.x, R = (NT + G - 1) / G;
    for (int r = 0; r < R; ++r) {
        const int t = NT - (r + 1) * G + blockIdx.x;
        if (t >= 0) rx_tile(y, iq, sym, t);
    }
}
__global__ __launch_bounds__(256) void k_fused(const uint4* bits, float4* y, float4* iq, unsigned* sym) {
    const int G = gridDim.x;
    int t = blockIdx.x;
    for (; t < NT; t += G) {
        tx_tile(bits, y, t);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t - G >= 0) rx_tile(y, iq, sym, t - G);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t - G < NT) rx_tile(y, iq, sym, t - G);
}
// lag 0: RX tile t right after TX tile t in the same workgroup (the tile just written)
__global__ __launch_bounds__(256) void k_fused0(const uint4* bits, float4* y, float4* iq, unsigned* sym) {
    for (int t = blockIdx.x; t < NT; t += gridDim.x) {
        tx_tile(bits, y, t);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        rx_tile(y, iq, sym, t);
    }
}
// the same with the TX tile stored write-through (sc1: the line leaves the XCD's L2)
typedef unsigned u4v __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_fused0_sc1(const uint4* bits, float4* y, float4* iq, unsigned* sym) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(y, 0, 0x7fffffff, 0x00020000);
    for (int t = blockIdx.x; t < NT; t += gridDim.x) {
        const uint4 b = bits[(size_t)t * 256 + threadIdx.x];
        const float v = (float)(b.x ^ b.y ^ b.z ^ b.w);
        const unsigned base = (unsigned)t * (TS * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j)
            __builtin_amdgcn_raw_buffer_store_b128((u4v){__float_as_uint(v), __float_as_uint(v + j), __float_as_uint(v),
                                                   __float_as_uint(v - j)}, r, base + (j * 256 + threadIdx.x) * 16, 0, 16);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        rx_tile(y, iq, sym, t);
    }
}
__global__ void k_wr(float4* o, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        o[i] = make_float4(1, 2, 3, 4);
}
__global__ void k_rd(const float4* x, float* o, size_t n) {
    float4 a = make_float4(0, 0, 0, 0);
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = x[i]; a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    if (a.x == 12345.f) o[0] = a.y + a.z + a.w;
}

static bool g_quick = false;                     // argv[1] == "pmc": 3 launches each, untimed
template <typename F> static void run(const char* name, double bytes, F f) {
    if (g_quick) { for (int i = 0; i < 3; ++i) f(); (void)hipDeviceSynchronize(); printf("%s\n", name); return; }
    for (int i = 0; i < 200; ++i) f();           // settle the clocks
    (void)hipDeviceSynchronize();
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    float best = 1e30f, sum = 0;
    const int R = 5, K = 200;
    for (int r = 0; r < R; ++r) {
        (void)hipEventRecord(a);
        for (int k = 0; k < K; ++k) f();
        (void)hipEventRecord(b); (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b); ms /= K;
        best = ms < best ? ms : best; sum += ms;
    }
    printf("%-44s min %7.2f us  mean %7.2f us  %6.2f TB/s (min)\n", name, best * 1e3, sum / R * 1e3,
           bytes / (best * 1e-3) / 1e12);
    fflush(stdout);
}

int main(int argc, char** argv) {
    g_quick = argc > 1 && argv[1][0] == 'p';
    uint4* bits; float4 *y, *iq; unsigned* sym; float* o;
    (void)hipMalloc(&bits, (size_t)NS); (void)hipMalloc(&y, (size_t)NS * 8);
    (void)hipMalloc(&iq, (size_t)NS / 4 * 8); (void)hipMalloc(&sym, (size_t)NS / 4); (void)hipMalloc(&o, 64);
    (void)hipMemset(bits, 1, (size_t)NS);
    const double btx = NS * 9.0, brx = NS * 8.0 + NS / 4 * 9.0, bch = btx + brx;
    int dev = 0, ncu = 0; (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    printf("CUs %d; chain bytes per period %.1f MB (19.25 B/sample)\n", ncu, bch / 1e6);
    for (int per : {2, 4, 8}) {
        const int G = ncu * per;
        char n[96];
        snprintf(n, 96, "two launches (tx; rx top-down) grid %d", G);
        run(n, bch, [&] { hipLaunchKernelGGL(k_tx, G, 256, 0, 0, bits, y);
                          hipLaunchKernelGGL(k_rx, G, 256, 0, 0, y, iq, sym); });
        snprintf(n, 96, "fused (tx t, rx t-G) grid %d", G);
        run(n, bch, [&] { hipLaunchKernelGGL(k_fused, G, 256, 0, 0, bits, y, iq, sym); });
        snprintf(n, 96, "fused lag 0 (tx t, rx t) grid %d", G);
        run(n, bch, [&] { hipLaunchKernelGGL(k_fused0, G, 256, 0, 0, bits, y, iq, sym); });
        snprintf(n, 96, "fused lag 0, tx sc1 stores grid %d", G);
        run(n, bch, [&] { hipLaunchKernelGGL(k_fused0_sc1, G, 256, 0, 0, bits, y, iq, sym); });
        snprintf(n, 96, "tx alone grid %d", G);
        run(n, btx, [&] { hipLaunchKernelGGL(k_tx, G, 256, 0, 0, bits, y); });
        snprintf(n, 96, "rx alone grid %d", G);
        run(n, brx, [&] { hipLaunchKernelGGL(k_rx, G, 256, 0, 0, y, iq, sym); });
    }
    const size_t n4 = (size_t)NS * 8 / 16;
    run("write 128 MiB + read 128 MiB (same buffer)", 2.0 * NS * 8, [&] {
        hipLaunchKernelGGL(k_wr, 2048, 256, 0, 0, y, n4);
        hipLaunchKernelGGL(k_rd, 2048, 256, 0, 0, y, o, n4); });
    return 0;
}
