// Tile-counter atomics on gfx950: one global counter (agent scope) vs one counter per XCD
// (workgroup-scope atomics on the XCD's L2), grabbed by every workgroup until N tiles are
// handed out. Checks that every tile index is handed out exactly once and times the grab loop.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
constexpr int N = 4096;
template <bool PER_XCD, bool WG_SCOPE>
__global__ void grab(unsigned* ctr, unsigned* seen, int spin) {
  __shared__ unsigned t;
  unsigned x = 0;
  if (PER_XCD) asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
  const unsigned lo = PER_XCD ? N / 8 * x : 0, hi = PER_XCD ? N / 8 * (x + 1) : N;
  float acc = 0.f;
  for (;;) {
    if (threadIdx.x == 0) {
      unsigned v = WG_SCOPE ? __hip_atomic_fetch_add(ctr + 64 * x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
                            : __hip_atomic_fetch_add(ctr + 64 * x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      t = lo + v;
    }
    __syncthreads();
    const unsigned tt = t;
    __syncthreads();
    if (tt >= hi) break;
    if (threadIdx.x == 0) atomicAdd(seen + tt, 1u);
    for (int i = 0; i < spin; ++i) acc = __builtin_fmaf(acc, 1.0001f, 0.5f);
  }
  if (acc == 1234.f) seen[N] = 1;
}
__global__ void stat(unsigned* ctr, unsigned* seen, int spin) {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
  if (threadIdx.x == 0) atomicAdd(ctr + 1024 + x, 1u);
  const unsigned t0 = N * blockIdx.x / gridDim.x, t1 = N * (blockIdx.x + 1) / gridDim.x;
  float acc = 0.f;
  for (unsigned tt = t0; tt < t1; ++tt) {
    if (threadIdx.x == 0) atomicAdd(seen + tt, 1u);
    for (int i = 0; i < spin; ++i) acc = __builtin_fmaf(acc, 1.0001f, 0.5f);
    __syncthreads();
  }
  if (acc == 1234.f) seen[N] = 1;
}
template <typename F> float timeit(F f) {
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a); f(); hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b); return ms * 1e3f;
}
int main() {
  unsigned *ctr, *seen;
  hipMalloc(&ctr, 2048 * 4); hipMalloc(&seen, (N + 1) * 4);
  std::vector<unsigned> h(N + 1);
  auto run = [&](const char* name, auto kern, int spin) {
    for (int rep = 0; rep < 3; ++rep) {
      hipMemset(ctr, 0, 2048 * 4); hipMemset(seen, 0, (N + 1) * 4); hipDeviceSynchronize();
      float us = timeit([&] { kern<<<768, 256>>>(ctr, seen, spin); });
      hipMemcpy(h.data(), seen, N * 4, hipMemcpyDeviceToHost);
      int miss = 0, dup = 0;
      for (int i = 0; i < N; ++i) { miss += h[i] == 0; dup += h[i] > 1; }
      unsigned wx[8]; hipMemcpy(wx, ctr + 1024, 32, hipMemcpyDeviceToHost);
      printf("%-34s spin %5d  %8.1f us  missing %d  duplicated %d", name, spin, us, miss, dup);
      if (rep == 0) { printf("  wg/xcd"); for (int i = 0; i < 8; ++i) printf(" %u", wx[i]); }
      printf("\n");
    }
  };
  for (int spin : {0, 2000}) {
    run("static ranges", stat, spin);
    run("global counter, agent scope", grab<false, false>, spin);
    run("per-XCD counter, agent scope", grab<true, false>, spin);
    run("per-XCD counter, workgroup scope", grab<true, true>, spin);
  }
  return 0;
}
