// Read bandwidth of the RX staging pattern on gfx950: persistent workgroups (256 lanes) walk
// contiguous ranges of 33.8-KB tiles (U = 5 x 32 B per lane per tile: two 16-B loads per slot),
// with D tiles in flight per workgroup (register double buffering), against a plain grid-stride
// float4 read. A fixed per-tile VALU cost (SPIN dependent FMAs per lane) stands in for staging.
// Build: hipcc -O3 --offload-arch=gfx950 rdtile.hip -o rdtile ; run on the GPU box.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#define NB (134217728ull)                 // bytes: 2^24 complex f32 samples
constexpr int NT = 256, U = 5;
constexpr size_t TILE = (size_t)NT * U * 32;   // 40960 B per tile

__global__ void rd4(const float4* x, float* o) {
  float a = 0;
  const size_t n = NB / 16;
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float4 v = x[i]; a += v.x + v.y + v.z + v.w;
  }
  if (a == 12345.f) o[0] = a;
}

template <int D, int SPIN, bool STRIDE>
__global__ __launch_bounds__(256) void tiles(const float4* x, float* o, int ntiles) {
  const int b = blockIdx.x, g = gridDim.x;
  int t0, t1, ts;
  if (STRIDE) { t0 = b; t1 = ntiles; ts = g; }
  else { t0 = (int)((long)ntiles * b / g); t1 = (int)((long)ntiles * (b + 1) / g); ts = 1; }
  float4 pre[D][U][2];
  auto load = [&](int t, int slot) {
    const float4* base = x + (size_t)t * (TILE / 16);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      pre[slot][u][0] = base[2 * (threadIdx.x + NT * u)];
      pre[slot][u][1] = base[2 * (threadIdx.x + NT * u) + 1];
    }
  };
#pragma unroll
  for (int d = 0; d < D; ++d) if (t0 + d * ts < t1) load(t0 + d * ts, d);
  float acc = 0.f;
  auto body = [&](int t, auto slot_c) {
    constexpr int slot = decltype(slot_c)::value;
    float s = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) s += pre[slot][u][0].x + pre[slot][u][1].w;
#pragma unroll
    for (int i = 0; i < SPIN; ++i) s = __builtin_fmaf(s, 1.0001f, 0.5f);
    acc += s;
    if (t + D * ts < t1) load(t + D * ts, slot);
    __syncthreads();
  };
  int t = t0;
  while (t < t1) {
    body(t, std::integral_constant<int, 0>()); t += ts;
    if (D > 1 && t < t1) { body(t, std::integral_constant<int, (D > 1 ? 1 : 0)>()); t += ts; }
    if (D > 2 && t < t1) { body(t, std::integral_constant<int, (D > 2 ? 2 : 0)>()); t += ts; }
  }
  if (acc == 12345.f) o[0] = acc;
}

template <typename F> void run(const char* name, F f) {
  f(); hipDeviceSynchronize();
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const int R = 20;
  hipEventRecord(a);
  for (int r = 0; r < R; ++r) f();
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  const double us = ms * 1e3 / R;
  printf("%-40s %8.2f us  %6.2f TB/s\n", name, us, NB / (us * 1e-6) / 1e12);
}

int main() {
  float4* x; float* o;
  hipMalloc(&x, NB + TILE); hipMalloc(&o, 64);
  hipMemset(x, 0, NB + TILE);
  const int ntiles = (int)(NB / TILE);
  run("rd4 grid-stride 4096x256", [&] { rd4<<<4096, 256>>>(x, o); });
#define T(D, S, ST, G) run("tiles D=" #D " spin=" #S " stride=" #ST " grid=" #G, \
    [&] { tiles<D, S, ST><<<G, 256>>>(x, o, ntiles); });
  T(1, 0, false, 768) T(2, 0, false, 768) T(3, 0, false, 768)
  T(1, 0, true, 768) T(2, 0, true, 768)
  T(1, 0, false, 1024) T(2, 0, false, 1024) T(1, 0, false, 1536)
  T(1, 400, false, 768) T(2, 400, false, 768)
  T(1, 800, false, 768) T(2, 800, false, 768)
  T(1, 1200, false, 768) T(2, 1200, false, 768) T(3, 1200, false, 512)
  T(1, 1200, true, 768) T(2, 1200, true, 768)
  return 0;
}
