// Streaming-bandwidth ceilings on gfx950 for the modem's access patterns (128 MiB buffers).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4v __attribute__((ext_vector_type(4)));
#define N4 (1 << 23)   // float4 elements = 128 MiB
__global__ void wr4(float4* o, float v) {
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < N4; i += gridDim.x * blockDim.x)
    o[i] = make_float4(v, v + 1, v + 2, v + 3);
}
__global__ void wr4nt(float4* o, float v) {
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < N4; i += gridDim.x * blockDim.x)
    __builtin_nontemporal_store((f4v){v, v + 1, v + 2, v + 3}, reinterpret_cast<f4v*>(o) + i);
}
__global__ void wr2(float2* o, float v) {
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < 2 * (size_t)N4; i += gridDim.x * blockDim.x)
    o[i] = make_float2(v, v + 1);
}
__global__ void rd4(const float4* x, float* o) {
  float4 a = {0, 0, 0, 0};
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < N4; i += gridDim.x * blockDim.x) {
    float4 v = x[i]; a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
  }
  if (a.x == 12345.f) o[0] = a.y + a.z + a.w;
}
// Each lane reads 32 contiguous bytes as two 16-B loads (lane stride 32 B), the RX quad pattern.
__global__ void rd8(const float4* x, float* o) {
  float4 a = {0, 0, 0, 0};
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; 2 * i < N4; i += gridDim.x * blockDim.x) {
    float4 v = x[2 * i], w = x[2 * i + 1];
    a.x += v.x + w.x; a.y += v.y + w.y; a.z += v.z + w.z; a.w += v.w + w.w;
  }
  if (a.x == 12345.f) o[0] = a.y + a.z + a.w;
}
// The same bytes with both loads coalesced (lane stride 16 B, second load 1 block later).
__global__ void rd8c(const float4* x, float* o) {
  float4 a = {0, 0, 0, 0};
  const size_t step = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * 2 * (size_t)blockDim.x + threadIdx.x; i < N4; i += 2 * step) {
    float4 v = x[i], w = x[i + blockDim.x];
    a.x += v.x + w.x; a.y += v.y + w.y; a.z += v.z + w.z; a.w += v.w + w.w;
  }
  if (a.x == 12345.f) o[0] = a.y + a.z + a.w;
}
__global__ void cp4(const float4* x, float4* o) {
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < N4; i += gridDim.x * blockDim.x) o[i] = x[i];
}
__global__ void wr4n(float4* o, float v, size_t n) {
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) o[i] = make_float4(v, v, v, v);
}
__global__ void rd4n(const float4* x, float* o, size_t n) {
  float4 a = make_float4(0, 0, 0, 0);
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const float4 v = x[i]; a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
  }
  if (a.x == 12345.f) o[0] = a.y + a.z + a.w;
}
template <typename F> void run(const char* name, double bytes, F f) {
  f(); hipDeviceSynchronize();
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const int R = 20;
  hipEventRecord(a); for (int r = 0; r < R; ++r) f(); hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b); ms /= R;
  printf("%-34s %8.1f us  %7.2f TB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
}
int main() {
  float4 *x, *y, *big; float* o;
  (void)hipMalloc(&x, (size_t)N4 * 16); (void)hipMalloc(&y, (size_t)N4 * 16); (void)hipMalloc(&o, 64);
  (void)hipMalloc(&big, (size_t)N4 * 16 * 4);
  (void)hipMemset(x, 0, (size_t)N4 * 16);
  const double B = (double)N4 * 16;
  for (int g : {1024, 2048, 4096}) {
    char n[64];
    snprintf(n, 64, "write float4 grid=%d", g); run(n, B, [&] { hipLaunchKernelGGL(wr4, g, 256, 0, 0, y, 1.f); });
    snprintf(n, 64, "write float4 nt grid=%d", g); run(n, B, [&] { hipLaunchKernelGGL(wr4nt, g, 256, 0, 0, y, 1.f); });
    snprintf(n, 64, "write float2 grid=%d", g); run(n, B, [&] { hipLaunchKernelGGL(wr2, g, 256, 0, 0, (float2*)y, 1.f); });
    snprintf(n, 64, "read float4 grid=%d", g); run(n, B, [&] { hipLaunchKernelGGL(rd4, g, 256, 0, 0, x, o); });
    snprintf(n, 64, "read 2xfloat4/lane stride32 g=%d", g); run(n, B, [&] { hipLaunchKernelGGL(rd8, g, 256, 0, 0, x, o); });
    snprintf(n, 64, "read 2xfloat4 coalesced g=%d", g); run(n, B, [&] { hipLaunchKernelGGL(rd8c, g, 256, 0, 0, x, o); });
    snprintf(n, 64, "copy float4 grid=%d", g); run(n, 2 * B, [&] { hipLaunchKernelGGL(cp4, g, 256, 0, 0, x, y); });
  }
  // write 128 MB then read it back (TX -> RX through the sample buffer): is the re-read L3-served?
  run("write128+read128 (same buf)", 2 * B, [&] {
    hipLaunchKernelGGL(wr4, 2048, 256, 0, 0, y, 1.f);
    hipLaunchKernelGGL(rd4, 2048, 256, 0, 0, y, o);
  });
  // 512 MiB (past the 256 MiB Infinity Cache): the HBM rates a C5 launch sees
  const size_t NB = (size_t)N4 * 4;
  for (int g : {2048, 4096}) {
    char n[64];
    snprintf(n, 64, "write 512MiB float4 grid=%d", g); run(n, 4 * B, [&] { hipLaunchKernelGGL(wr4n, g, 256, 0, 0, big, 1.f, NB); });
    snprintf(n, 64, "read 512MiB float4 grid=%d", g); run(n, 4 * B, [&] { hipLaunchKernelGGL(rd4n, g, 256, 0, 0, big, o, NB); });
  }
  run("write512+read512 (same buf)", 8 * B, [&] {
    hipLaunchKernelGGL(wr4n, 4096, 256, 0, 0, big, 1.f, NB);
    hipLaunchKernelGGL(rd4n, 4096, 256, 0, 0, big, o, NB);
  });
  return 0;
}
