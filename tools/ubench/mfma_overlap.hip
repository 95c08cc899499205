// Does v_mfma_f32_16x16x4_f32 from one wave overlap with packed-VALU work of another wave
// on the same SIMD (gfx950)? Compare MFMA-only, VALU-only and mixed kernels (same per-wave
// work); 8 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
#define IT 2048
__device__ __forceinline__ void mfma_work(float* o, int lane) {
  f32x4 a0 = {0, 0, 0, 0}, a1 = a0, a2 = a0, a3 = a0;
  float x = lane * 1e-3f, y = 1.0001f;
  for (int i = 0; i < IT; ++i) {
    a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x, y, a0, 0, 0, 0);
    a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(y, x, a1, 0, 0, 0);
    a2 = __builtin_amdgcn_mfma_f32_16x16x4f32(x, x, a2, 0, 0, 0);
    a3 = __builtin_amdgcn_mfma_f32_16x16x4f32(y, y, a3, 0, 0, 0);
  }
  o[lane] = a0[0] + a1[1] + a2[2] + a3[3];
}
__device__ __forceinline__ void valu_work(float* o, int lane) {
  f2 v[16]; for (int i = 0; i < 16; ++i) v[i] = (f2){lane * 1e-3f + i, 1.f * i};
  for (int i = 0; i < IT; ++i) {
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = __builtin_elementwise_fma(v[k], (f2){0.999f, 0.999f}, (f2){0.5f, 0.25f});
  }
  float t = 0; for (int k = 0; k < 16; ++k) t += v[k].x + v[k].y; o[lane] = t;
}
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
// f16 inputs, f32 accumulate: 16x16x32 (8192 MACs, ~16 cyc) — the matrix cores proper.
// 8 per iteration (8 x 16 cyc) to match the f32 variant's per-iteration cost.
__device__ __forceinline__ void mfma16_work(float* o, int lane) {
  f32x4 a0 = {0, 0, 0, 0}, a1 = a0, a2 = a0, a3 = a0;
  h8 x, y;
  for (int k = 0; k < 8; ++k) { x[k] = (_Float16)(lane * 1e-3f + k); y[k] = (_Float16)1.0f; }
  for (int i = 0; i < IT; ++i) {
    a0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(x, y, a0, 0, 0, 0);
    a1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(y, x, a1, 0, 0, 0);
    a2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(x, x, a2, 0, 0, 0);
    a3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(y, y, a3, 0, 0, 0);
    a0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(x, y, a0, 0, 0, 0);
    a1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(y, x, a1, 0, 0, 0);
    a2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(x, x, a2, 0, 0, 0);
    a3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(y, y, a3, 0, 0, 0);
  }
  o[lane] = a0[0] + a1[1] + a2[2] + a3[3];
}
// 4 MFMA (4 x 32 cyc) per iteration vs 16 pk_fma (16 x ~4.5 cyc): similar per-iteration cost.
__global__ void k_mfma(float* o) { mfma_work(o + blockIdx.x * 64, threadIdx.x & 63); }
__global__ void k_valu(float* o) { valu_work(o + blockIdx.x * 64, threadIdx.x & 63); }
__global__ void k_mixed(float* o) {   // waves 0-3 (one per SIMD) MFMA, waves 4-7 VALU
  if ((threadIdx.x >> 6) < 4) mfma_work(o + blockIdx.x * 64, threadIdx.x & 63);
  else valu_work(o + blockIdx.x * 64, threadIdx.x & 63);
}
__global__ void k_mfma16(float* o) { mfma16_work(o + blockIdx.x * 64, threadIdx.x & 63); }
__global__ void k_mixed16(float* o) {   // waves 0-3 f16 MFMA, waves 4-7 VALU
  if ((threadIdx.x >> 6) < 4) mfma16_work(o + blockIdx.x * 64, threadIdx.x & 63);
  else valu_work(o + blockIdx.x * 64, threadIdx.x & 63);
}
template <typename F> float run(const char* name, F f) {
  f(); hipDeviceSynchronize();
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a); for (int r = 0; r < 5; ++r) f(); hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b); ms /= 5;
  printf("%-40s %8.3f ms\n", name, ms);
  return ms;
}
int main() {
  float* o; (void)hipMalloc(&o, 1 << 24);
  const int B = 256 * 4;   // 4 workgroups of 512 threads per CU -> 8 waves/SIMD
  run("MFMA only (512-thr blocks)", [&] { hipLaunchKernelGGL(k_mfma, B, 512, 0, 0, o); });
  run("VALU only (512-thr blocks)", [&] { hipLaunchKernelGGL(k_valu, B, 512, 0, 0, o); });
  run("half MFMA waves + half VALU waves", [&] { hipLaunchKernelGGL(k_mixed, B, 512, 0, 0, o); });
  run("MFMA only, half the waves", [&] { hipLaunchKernelGGL(k_mfma, B, 256, 0, 0, o); });
  run("VALU only, half the waves", [&] { hipLaunchKernelGGL(k_valu, B, 256, 0, 0, o); });
  run("f16 MFMA only (512-thr blocks)", [&] { hipLaunchKernelGGL(k_mfma16, B, 512, 0, 0, o); });
  run("f16 MFMA only, half the waves", [&] { hipLaunchKernelGGL(k_mfma16, B, 256, 0, 0, o); });
  run("half f16-MFMA waves + half VALU waves", [&] { hipLaunchKernelGGL(k_mixed16, B, 512, 0, 0, o); });
  return 0;
}
