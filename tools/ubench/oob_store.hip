// Probe (round 6): how a raw buffer store of two dwords that is only partly inside the descriptor's
// records behaves on gfx950 — are the in-range dword(s) written or the whole store dropped? Decides
// whether the RX's f16 pair stores (two instants per lane, whole 128-B lines) may straddle the end of
// a call's instants. Build: hipcc -O2 --offload-arch=gfx950 oob_store.hip -o oob_store
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u2 __attribute__((ext_vector_type(2)));

__device__ __amdgpu_buffer_rsrc_t rsrc(void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(base, 0, bytes, 0x00020000);
}

__global__ void probe(uint32_t* out) {
    if (threadIdx.x != 0) return;
    // case 0: dwordx2 at offset 0, records 4: dword 0 in range, dword 1 out
    __builtin_amdgcn_raw_buffer_store_b64((u2){0xA0, 0xA1}, rsrc(out + 0, 4), 0, 0, 0);
    // case 1: dwordx2 at offset 4, records 8: dword 0 (byte 4) in range, dword 1 (byte 8) out
    __builtin_amdgcn_raw_buffer_store_b64((u2){0xB0, 0xB1}, rsrc(out + 4, 8), 4, 0, 0);
    // case 2: dwordx2 at offset 0xFFFFFFFC (a wrapped -4), records 8: dword 1 would land at byte 0
    __builtin_amdgcn_raw_buffer_store_b64((u2){0xC0, 0xC1}, rsrc(out + 9, 8), 0xFFFFFFFCu, 0, 0);
    // case 3: control, fully in range
    __builtin_amdgcn_raw_buffer_store_b64((u2){0xD0, 0xD1}, rsrc(out + 12, 8), 0, 0, 0);
    // case 4: dwordx4 at offset 0, records 8: dwords 0-1 in, 2-3 out
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    __builtin_amdgcn_raw_buffer_store_b128((u4){0xE0, 0xE1, 0xE2, 0xE3}, rsrc(out + 16, 8), 0, 0, 0);
    // case 5: one dword straddling the end of the records (records 2: bytes 0-1 in range)
    __builtin_amdgcn_raw_buffer_store_b32(0x44332211u, rsrc(out + 20, 2), 0, 0, 0);
    // case 6: dwordx2 whose second dword straddles the end (records 6)
    __builtin_amdgcn_raw_buffer_store_b64((u2){0x88776655u, 0xCCBBAA99u}, rsrc(out + 22, 6), 0, 0, 0);
}

int main() {
    uint32_t* d;
    const int n = 28;
    if (hipMalloc(&d, n * 4) != hipSuccess) return 1;
    hipMemset(d, 0, n * 4);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
    uint32_t h[n];
    if (hipMemcpy(h, d, n * 4, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    printf("case0 (x2 at 0, records 4):       [0]=%x [1]=%x\n", h[0], h[1]);
    printf("case1 (x2 at 4, records 8):       [5]=%x [6]=%x\n", h[5], h[6]);
    printf("case2 (x2 at -4, records 8):      [8]=%x [9]=%x\n", h[8], h[9]);
    printf("case3 (control):                  [12]=%x [13]=%x\n", h[12], h[13]);
    printf("case4 (x4 at 0, records 8):       [16]=%x [17]=%x [18]=%x [19]=%x\n", h[16], h[17], h[18], h[19]);
    printf("case5 (x1 straddling, records 2): [20]=%08x\n", h[20]);
    printf("case6 (x2, records 6):            [22]=%08x [23]=%08x\n", h[22], h[23]);
    hipFree(d);
    return 0;
}
