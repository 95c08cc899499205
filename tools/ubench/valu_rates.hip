// Microbenchmark: per-wave issue cost of the VALU ops the modem kernels lean on (gfx950).
// Each kernel runs ITERS x 16 independent ops per lane; time / ops gives cycles per op per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <chrono>
typedef float f2 __attribute__((ext_vector_type(2)));
#define ITERS 4096
__global__ void k_fma(float* o, float s) {
  float a[16]; for (int i = 0; i < 16; ++i) a[i] = threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = __builtin_fmaf(a[i], s, 0.5f);
  }
  float t = 0; for (int i = 0; i < 16; ++i) t += a[i]; o[blockIdx.x * blockDim.x + threadIdx.x] = t;
}
__global__ void k_pkfma(float* o, float s) {
  f2 a[16]; for (int i = 0; i < 16; ++i) a[i] = (f2){(float)threadIdx.x + i, 1.0f * i};
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = __builtin_elementwise_fma(a[i], (f2){s, s}, (f2){0.5f, 0.25f});
  }
  float t = 0; for (int i = 0; i < 16; ++i) t += a[i].x + a[i].y; o[blockIdx.x * blockDim.x + threadIdx.x] = t;
}
__global__ void k_sin(float* o, float s) {
  float a[16]; for (int i = 0; i < 16; ++i) a[i] = threadIdx.x * 1e-3f + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = __builtin_amdgcn_sinf(a[i]);
  }
  float t = 0; for (int i = 0; i < 16; ++i) t += a[i]; o[blockIdx.x * blockDim.x + threadIdx.x] = t;
}
__global__ void k_lds(float* o, int stride) {
  __shared__ float2 sm[8192];
  for (int i = threadIdx.x; i < 8192; i += blockDim.x) sm[i] = make_float2(i, i);
  __syncthreads();
  f2 acc = {0, 0};
  int base = (threadIdx.x * stride) & 4095;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) { float2 v = sm[base + i * 64]; acc += (f2){v.x, v.y}; }
    base ^= 1;
  }
  o[blockIdx.x * blockDim.x + threadIdx.x] = acc.x + acc.y;
}
// 16 independent fma + 4 independent v_sin per iteration: does the transcendental unit
// overlap the FMA pipe (time ~ max) or share it (time ~ sum)?
__global__ void k_fma_sin(float* o, float s) {
  float a[16], b[4]; for (int i = 0; i < 16; ++i) a[i] = threadIdx.x + i;
  for (int i = 0; i < 4; ++i) b[i] = threadIdx.x * 1e-3f + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = __builtin_fmaf(a[i], s, 0.5f);
#pragma unroll
    for (int i = 0; i < 4; ++i) b[i] = __builtin_amdgcn_sinf(b[i]);
  }
  float t = 0; for (int i = 0; i < 16; ++i) t += a[i]; for (int i = 0; i < 4; ++i) t += b[i];
  o[blockIdx.x * blockDim.x + threadIdx.x] = t;
}
// dependent chains (latency): 2 independent chains per lane
__global__ void k_fma_dep(float* o, float s) {
  float a = threadIdx.x, b = threadIdx.x + 1;
  for (int it = 0; it < ITERS * 8; ++it) { a = __builtin_fmaf(a, s, 0.5f); b = __builtin_fmaf(b, s, 0.25f); }
  o[blockIdx.x * blockDim.x + threadIdx.x] = a + b;
}
__global__ void k_pkfma_dep(float* o, float s) {
  f2 a = {(float)threadIdx.x, 1.f}, b = {2.f, (float)threadIdx.x};
  for (int it = 0; it < ITERS * 8; ++it) {
    a = __builtin_elementwise_fma(a, (f2){s, s}, (f2){0.5f, 0.25f});
    b = __builtin_elementwise_fma(b, (f2){s, s}, (f2){0.5f, 0.25f});
  }
  o[blockIdx.x * blockDim.x + threadIdx.x] = a.x + a.y + b.x + b.y;
}
__global__ void k_floor(float* o, float s) {
  float a[16]; for (int i = 0; i < 16; ++i) a[i] = threadIdx.x * 0.37f + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = __builtin_floorf(a[i] * s);
  }
  float t = 0; for (int i = 0; i < 16; ++i) t += a[i]; o[blockIdx.x * blockDim.x + threadIdx.x] = t;
}
// v_fma_mix_f32 with an f16 first source (the conversion folded into the FMA) and the plain
// v_cvt_f32_f16 it would replace: issue cost of each (asm, so the forms are exactly these)
__global__ void k_fmamix(float* o, float s) {
  float a[16]; for (int i = 0; i < 16; ++i) a[i] = threadIdx.x + i;
  const uint32_t h = 0x3c003c00u + threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(a[i]) : "v"(h), "v"(s));
  }
  float t = 0; for (int i = 0; i < 16; ++i) t += a[i]; o[blockIdx.x * blockDim.x + threadIdx.x] = t;
}
__global__ void k_cvt(float* o, float s) {
  float a[16]; uint32_t h[16];
  for (int i = 0; i < 16; ++i) { a[i] = 0; h[i] = 0x3c003c00u + threadIdx.x + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) asm volatile("v_cvt_f32_f16 %0, %1" : "=v"(a[i]) : "v"(h[i]));
  }
  float t = 0; for (int i = 0; i < 16; ++i) t += a[i]; o[blockIdx.x * blockDim.x + threadIdx.x] = t;
}
template <typename F> double run(F f, const char* name, double ops_per_lane, int blocks, int threads) {
  float* o; hipMalloc(&o, (size_t)blocks * threads * 4);
  f(o); hipDeviceSynchronize();
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a); for (int r = 0; r < 5; ++r) f(o); hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b); ms /= 5;
  int dev; hipGetDevice(&dev); int clk; hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
  double waves = (double)blocks * threads / 64, simds = 256 * 4;
  double wave_ops = waves * ops_per_lane;                 // wave-instructions
  double cyc = ms * 1e-3 * clk * 1e3;                     // at the reported max clock
  printf("%-28s %8.3f ms  %.2f cycles per wave-op per SIMD (at %d MHz)\n", name, ms, cyc * simds / wave_ops, clk / 1000);
  hipFree(o); return ms;
}
int main() {
  for (int occ = 4; occ <= 8; occ += 4) {
  const int B = 256 * occ, T = 256;   // occ waves / SIMD
  printf("== %d waves per SIMD\n", occ);
  run([&](float* o) { hipLaunchKernelGGL(k_fma_sin, B, T, 0, 0, o, 0.999f); }, "16 fma + 4 sin (per 16 fma)", ITERS * 16.0, B, T);
  run([&](float* o) { hipLaunchKernelGGL(k_fma_dep, B, T, 0, 0, o, 0.999f); }, "v_fma_f32 2 dep chains", ITERS * 16.0, B, T);
  run([&](float* o) { hipLaunchKernelGGL(k_pkfma_dep, B, T, 0, 0, o, 0.999f); }, "v_pk_fma_f32 2 dep chains", ITERS * 16.0, B, T);
  run([&](float* o) { hipLaunchKernelGGL(k_floor, B, T, 0, 0, o, 0.999f); }, "v_mul+v_floor (per pair)", ITERS * 16.0, B, T);
  run([&](float* o) { hipLaunchKernelGGL(k_fma, B, T, 0, 0, o, 0.999f); }, "v_fma_f32", ITERS * 16.0, B, T);
  run([&](float* o) { hipLaunchKernelGGL(k_pkfma, B, T, 0, 0, o, 0.999f); }, "v_pk_fma_f32", ITERS * 16.0, B, T);
  run([&](float* o) { hipLaunchKernelGGL(k_sin, B, T, 0, 0, o, 0.999f); }, "v_sin_f32", ITERS * 16.0, B, T);
  run([&](float* o) { hipLaunchKernelGGL(k_fmamix, B, T, 0, 0, o, 0.999f); }, "v_fma_mix_f32 (f16 src0)", ITERS * 16.0, B, T);
  run([&](float* o) { hipLaunchKernelGGL(k_cvt, B, T, 0, 0, o, 0.999f); }, "v_cvt_f32_f16", ITERS * 16.0, B, T);
  run([&](float* o) { hipLaunchKernelGGL(k_lds, B / 2, T, 0, 0, o, 1); }, "ds_read_b64 stride8B(+add)", ITERS * 16.0, B / 2, T);
  run([&](float* o) { hipLaunchKernelGGL(k_lds, B / 2, T, 0, 0, o, 2); }, "ds_read_b64 stride16B(+add)", ITERS * 16.0, B / 2, T);
  run([&](float* o) { hipLaunchKernelGGL(k_lds, B / 2, T, 0, 0, o, 5); }, "ds_read_b64 stride40B(+add)", ITERS * 16.0, B / 2, T);
  }
  return 0;
}
