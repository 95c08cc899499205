// FETCH_SIZE calibration by load width. MI355X_MICROARCH.md: on gfx950
// FETCH_SIZE reports half the bytes of a 16-B-per-lane streaming read; the TX reads its bits
// 4 B (C3, 4 bits per symbol) or 8 B (C5) per lane. Each kernel reads exactly 64 MiB once,
// lanes at consecutive addresses (the TX's symbol-per-lane pattern), one launch per width, so
// that a `rocprofv3 --pmc FETCH_SIZE` pass gives bytes / (FETCH_SIZE KiB * 1024) per width.
//
// hipcc -O3 --offload-arch=gfx950 fetch_cal.hip -o fetch_cal
// rocprofv3 --pmc FETCH_SIZE --output-format csv -d <dir> -o run -- ./fetch_cal
#include <hip/hip_runtime.h>
#include <cstdio>

#define BYTES (64u << 20)

template <typename W>
__global__ __launch_bounds__(256) void rd(const W* __restrict__ x, unsigned* __restrict__ o) {
    const size_t n = BYTES / sizeof(W);
    unsigned a = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const W v = x[i];
        a ^= reinterpret_cast<const unsigned*>(&v)[0];
    }
    if (a == 0x12345679u) o[0] = a;
}

int main() {
    char* x; unsigned* o; char* flush;
    (void)hipMalloc(&x, BYTES); (void)hipMalloc(&o, 64); (void)hipMalloc(&flush, 512u << 20);
    (void)hipMemset(x, 1, BYTES);
    for (int rep = 0; rep < 3; ++rep) {
        // 512 MiB written between the reads: nothing of x stays in the L2s or the Infinity Cache
        (void)hipMemset(flush, rep, 512u << 20);
        hipLaunchKernelGGL((rd<unsigned>), 2048, 256, 0, 0, (const unsigned*)x, o);          // 4 B / lane
        (void)hipMemset(flush, rep + 1, 512u << 20);
        hipLaunchKernelGGL((rd<uint2>), 2048, 256, 0, 0, (const uint2*)x, o);                // 8 B / lane
        (void)hipMemset(flush, rep + 2, 512u << 20);
        hipLaunchKernelGGL((rd<uint4>), 2048, 256, 0, 0, (const uint4*)x, o);                // 16 B / lane
        (void)hipMemset(flush, rep + 3, 512u << 20);
        hipLaunchKernelGGL((rd<unsigned char>), 2048, 256, 0, 0, (const unsigned char*)x, o); // 1 B / lane
    }
    (void)hipDeviceSynchronize();
    printf("fetch_cal: each rd<W> launch reads %u bytes\n", BYTES);
    return 0;
}
