// Layout probe: v_mfma_f64_16x16x4_f64 vs v_mfma_f32_16x16x4_f32 operand/result lane mapping.
// A[i][k] = 1000 + 10*i + k... use values that identify (i,k): A = i + 100*k, B = identity-like.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void probe(double *out64, float *out32) {
    const int l = threadIdx.x, i = l & 15, k = l >> 4;
    // A[i][k] = i + 16*k (lane l supplies A[l&15][l>>4]); B[k][j] = (k == 0) ? 1 : 0 (lane supplies B[l>>4][l&15])
    (void)i; (void)k;
    const double a = (double)((l * 37 + 11) % 101) - 50.0, b = (double)((l * 53 + 5) % 97) - 48.0;  // exact ints
    d4 acc = {0, 0, 0, 0};
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    f4 acc32 = {0, 0, 0, 0};
    acc32 = __builtin_amdgcn_mfma_f32_16x16x4f32((float)a, (float)b, acc32, 0, 0, 0);
    for (int r = 0; r < 4; ++r) { out64[l * 4 + r] = acc[r]; out32[l * 4 + r] = acc32[r]; }
}
int main() {
    double *d64; float *d32;
    hipMalloc(&d64, 256 * 8); hipMalloc(&d32, 256 * 4);
    hipLaunchKernelGGL(probe, 1, 64, 0, 0, d64, d32);
    double h64[256]; float h32[256];
    hipMemcpy(h64, d64, sizeof h64, hipMemcpyDeviceToHost);
    hipMemcpy(h32, d32, sizeof h32, hipMemcpyDeviceToHost);
    // D[i][j] = sum_k A[i][k] B[k][j] = A[i][0] = i  (for every j)
    int bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 4; ++r) {
            if (h64[l * 4 + r] != (double)h32[l * 4 + r]) bad++;
            if (l < 20 || h64[l*4+r] != (double)h32[l*4+r]) if (r == 0 && l % 8 == 0) printf("lane %2d r%d f64 %g f32 %g\n", l, r, h64[l*4+r], h32[l*4+r]);
        }
    // second probe: identify row/col: B[k][j] = j+1 when k==0
    printf("mismatches %d\n", bad);
    for (int l = 0; l < 64; ++l) printf("F64 %d %g %g %g %g\n", l, h64[l*4], h64[l*4+1], h64[l*4+2], h64[l*4+3]);
    return 0;
}
