// Unit check of the inline-asm helpers used by the RX staging (packed conjugate mix,
// v_fma_mix_f32 split remainder, v_max3 with |.|) against plain C on the host.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
typedef float cf2 __attribute__((ext_vector_type(2)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ cf2 cmix(cf2 x, cf2 cssn) {
    cf2 t, z;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(t) : "v"(x), "v"(cssn));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[0,1,0]"
        : "=v"(z) : "v"(x), "v"(cssn), "v"(t));
    return z;
}
__global__ void k(const float* in, float* out, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float x = in[4 * i], y = in[4 * i + 1], cs = in[4 * i + 2], sn = in[4 * i + 3];
    cf2 z = cmix((cf2){x, y}, (cf2){cs, sn});
    h2 hi = __builtin_convertvector((cf2){x, y}, h2);
    float l0, l1;
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(l0) : "v"(hi), "v"(x));
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(l1) : "v"(hi), "v"(y));
    float mx = 0.25f;
    asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(mx) : "v"(x), "v"(y));
    out[8 * i] = z.x; out[8 * i + 1] = z.y; out[8 * i + 2] = l0; out[8 * i + 3] = l1; out[8 * i + 4] = mx;
    out[8 * i + 5] = (float)hi.x; out[8 * i + 6] = (float)hi.y;
}
int main() {
    const int n = 4096;
    float* h = new float[4 * n]; float* r = new float[8 * n];
    unsigned s = 12345;
    for (int i = 0; i < 4 * n; ++i) { s = s * 1664525u + 1013904223u; h[i] = ((s >> 8) / 16777216.0f - 0.5f) * 4.0f; }
    float *din, *dout; (void)hipMalloc(&din, 16 * n); (void)hipMalloc(&dout, 32 * n);
    (void)hipMemcpy(din, h, 16 * n, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, n / 256, 256, 0, 0, din, dout, n);
    (void)hipMemcpy(r, dout, 32 * n, hipMemcpyDeviceToHost);
    int bad[4] = {0, 0, 0, 0};
    for (int i = 0; i < n; ++i) {
        float x = h[4*i], y = h[4*i+1], cs = h[4*i+2], sn = h[4*i+3];
        float zr = std::fma(y, sn, x * cs), zi = std::fma(-x, sn, y * cs);
        float hx = r[8*i+5], hy = r[8*i+6];
        float mx = std::fmax(0.25f, std::fmax(std::fabs(x), std::fabs(y)));
        if (r[8*i] != zr || r[8*i+1] != zi) { if (bad[0]++ < 3) printf("mix %d: got %g %g want %g %g\n", i, r[8*i], r[8*i+1], zr, zi); }
        if (r[8*i+2] != x - hx || r[8*i+3] != y - hy) { if (bad[1]++ < 3) printf("rem %d: got %g %g want %g %g\n", i, r[8*i+2], r[8*i+3], x - hx, y - hy); }
        if (r[8*i+4] != mx) { if (bad[2]++ < 3) printf("max %d: got %g want %g\n", i, r[8*i+4], mx); }
    }
    printf("mismatches: mix %d, split remainder %d, max3 %d (of %d)\n", bad[0], bad[1], bad[2], n);
    return bad[0] || bad[1] || bad[2];
}
