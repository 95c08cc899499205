// WRITE_SIZE calibration by store width and pattern (round 6). MI355X_MICROARCH.md:
// WRITE_SIZE reads the bytes exactly for 16-B-per-lane streaming stores; other widths are uncalibrated.
// The RX writes its decisions one byte per lane (16 B per 16-lane row, the MFMA output layout) and
// f16 I/Q four bytes per lane. Each kernel writes exactly 8 MiB once (one launch per pattern), so
// that a `rocprofv3 --pmc WRITE_SIZE` pass gives WRITE_SIZE KiB * 1024 / bytes per pattern:
//   st_b8_rows   the RX decision pattern: per wave block of 256 B, lane (c, g) writes byte
//                64 g + 16 r + c for r = 0..3 (four b8 stores per lane)
//   st_b32_lin   4 B per lane, each wave instruction 256 contiguous bytes
//   st_b32_rows  the RX f16 I/Q pattern: per 1 KiB block, lane (c, g) writes 4 B at instant
//                64 g + 16 r + c for r = 0..3
//   st_b128_lin  16 B per lane (the calibrated reference)
//
// hipcc -O3 --offload-arch=gfx950 write_cal.hip -o write_cal
// rocprofv3 --pmc WRITE_SIZE --output-format csv -d <dir> -o run -- ./write_cal
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define BYTES (8u << 20)

__global__ __launch_bounds__(256) void st_b8_rows(uint8_t* __restrict__ y) {
    const unsigned lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
    for (size_t blk = (blockIdx.x * 4 + (threadIdx.x >> 6)); blk < BYTES / 256; blk += gridDim.x * 4)
#pragma unroll
        for (int r = 0; r < 4; ++r) y[blk * 256 + 64 * g + 16 * r + c] = (uint8_t)(r + c);
}

__global__ __launch_bounds__(256) void st_b32_lin(uint32_t* __restrict__ y) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < BYTES / 4; i += (size_t)gridDim.x * blockDim.x)
        y[i] = (uint32_t)i;
}

__global__ __launch_bounds__(256) void st_b32_rows(uint32_t* __restrict__ y) {
    const unsigned lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
    for (size_t blk = (blockIdx.x * 4 + (threadIdx.x >> 6)); blk < BYTES / 1024; blk += gridDim.x * 4)
#pragma unroll
        for (int r = 0; r < 4; ++r) y[blk * 256 + 64 * g + 16 * r + c] = (uint32_t)(r + c);
}

__global__ __launch_bounds__(256) void st_b128_lin(uint4* __restrict__ y) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < BYTES / 16; i += (size_t)gridDim.x * blockDim.x)
        y[i] = make_uint4((unsigned)i, 1u, 2u, 3u);
}

int main() {
    char* y; char* flush;
    (void)hipMalloc(&y, BYTES); (void)hipMalloc(&flush, 512u << 20);
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipMemset(flush, rep, 512u << 20);
        hipLaunchKernelGGL(st_b8_rows, 1024, 256, 0, 0, (uint8_t*)y);
        (void)hipMemset(flush, rep + 1, 512u << 20);
        hipLaunchKernelGGL(st_b32_lin, 1024, 256, 0, 0, (uint32_t*)y);
        (void)hipMemset(flush, rep + 2, 512u << 20);
        hipLaunchKernelGGL(st_b32_rows, 1024, 256, 0, 0, (uint32_t*)y);
        (void)hipMemset(flush, rep + 3, 512u << 20);
        hipLaunchKernelGGL(st_b128_lin, 1024, 256, 0, 0, (uint4*)y);
    }
    (void)hipDeviceSynchronize();
    printf("write_cal: each launch writes %u bytes\n", BYTES);
    return 0;
}
