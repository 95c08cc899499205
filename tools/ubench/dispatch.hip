// Microbenchmark: how fast does a persistent grid get dispatched on gfx950? Each wave stores
// s_memrealtime (100 MHz) at entry; the spread first -> last entry per configuration, for the
// RX kernel's resource shape (256-thread workgroups, ~120 VGPRs, ~106 SGPRs, ~37 KB LDS, 4 per
// CU) against lighter shapes and fewer, wider workgroups.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

template <int VG, int SG>
__global__ void k_entry(unsigned long long* t, int spin) {
  extern __shared__ float lds[];
  const unsigned long long r = __builtin_amdgcn_s_memrealtime();
  if (VG > 64) asm volatile("v_mov_b32 v119, 0" ::: "v119");
  if (SG > 64) asm volatile("s_mov_b32 s100, 0" ::: "s100");
  if ((threadIdx.x & 63) == 0) t[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = r;
  // keep the workgroup resident for `spin` us so that the grid is persistent-like
  const unsigned long long end = r + (unsigned long long)spin * 100;
  while (__builtin_amdgcn_s_memrealtime() < end) __builtin_amdgcn_s_sleep(2);
  if (spin < 0) lds[threadIdx.x] = 1.f;
}

template <int VG, int SG>
void run(const char* name, int blocks, int threads, size_t lds, int spin) {
  const int waves = blocks * threads / 64;
  unsigned long long* d;
  hipMalloc(&d, waves * 8);
  std::vector<unsigned long long> h(waves);
  double sp[3];
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  float ms = 0;
  for (int rep = 0; rep < 4; ++rep) {
    hipEventRecord(a);
    hipLaunchKernelGGL((k_entry<VG, SG>), dim3(blocks), dim3(threads), lds, 0, d, spin);
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    hipMemcpy(h.data(), d, waves * 8, hipMemcpyDeviceToHost);
    auto mm = std::minmax_element(h.begin(), h.end());
    if (rep) sp[rep - 1] = (*mm.second - *mm.first) / 100.0;
  }
  printf("%-44s blocks %5d x %4d lds %6zu  entry spread %.2f %.2f %.2f us  kernel %.2f us\n", name, blocks, threads,
         lds, sp[0], sp[1], sp[2], ms * 1e3);
  hipFree(d);
}

int main() {
  const int spin = 20;   // us resident
  run<8, 8>("light 256-thr", 1024, 256, 0, spin);
  run<8, 8>("light 256-thr + 37 KB LDS", 1024, 256, 37888, spin);
  run<120, 8>("120 VGPR 256-thr", 1024, 256, 0, spin);
  run<120, 106>("120 VGPR 106 SGPR 256-thr + 37 KB LDS", 1024, 256, 37888, spin);
  run<120, 106>("RX shape x 5/4 (oversubscribed)", 1280, 256, 37888, spin);
  run<120, 106>("512-thr, 2 per CU, 74 KB", 512, 512, 75776, spin);
  run<120, 106>("1024-thr, 1 per CU, 148 KB", 256, 1024, 151552, spin);
  run<8, 8>("light 64-thr x 4096", 4096, 64, 0, spin);
  return 0;
}
