// Layout + timing probe of v_mfma_f32_4x4x1_16b_f32 (gfx950), for the narrow output layer:
// hypothesis: lane l is block b = l / 4 with A_b[l % 4][0] = a_l, B_b[0][l % 4] = b_l, and D lane
// 4b + j register i = sum over the chained instructions of A_b[i] * B_b[j].
// Timing: dependent chains of 64 instructions, 4x4x1 vs 16x16x4 (s_memtime).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void probe(const float *a, const float *b, float *out, long long *cyc) {
    const int l = threadIdx.x;
    f4 acc = {0, 0, 0, 0};
    for (int s = 0; s < 3; ++s) acc = __builtin_amdgcn_mfma_f32_4x4x1f32(a[s * 64 + l], b[s * 64 + l], acc, 0, 0, 0);
    for (int r = 0; r < 4; ++r) out[l * 4 + r] = acc[r];
    f4 x = {1, 1, 1, 1}, y = {1, 1, 1, 1};
    const float u = a[l] * 1e-3f, v = b[l] * 1e-3f;
    __builtin_amdgcn_sched_barrier(0);
    long long t0 = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < 64; ++k) x = __builtin_amdgcn_mfma_f32_4x4x1f32(u, v, x, 0, 0, 0);
    asm volatile("" ::"v"(x));
    __builtin_amdgcn_sched_barrier(0);
    long long t1 = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < 64; ++k) y = __builtin_amdgcn_mfma_f32_16x16x4f32(u, v, y, 0, 0, 0);
    asm volatile("" ::"v"(y));
    __builtin_amdgcn_sched_barrier(0);
    long long t2 = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
    f4 p = {1, 1, 1, 1}, q = {1, 1, 1, 1}, r2 = {1, 1, 1, 1}, s2 = {1, 1, 1, 1};
#pragma unroll
    for (int k = 0; k < 16; ++k) {       // 4 independent 4x4x1 chains: throughput
        p = __builtin_amdgcn_mfma_f32_4x4x1f32(u, v, p, 0, 0, 0);
        q = __builtin_amdgcn_mfma_f32_4x4x1f32(u, v, q, 0, 0, 0);
        r2 = __builtin_amdgcn_mfma_f32_4x4x1f32(u, v, r2, 0, 0, 0);
        s2 = __builtin_amdgcn_mfma_f32_4x4x1f32(u, v, s2, 0, 0, 0);
    }
    asm volatile("" ::"v"(p), "v"(q), "v"(r2), "v"(s2));
    __builtin_amdgcn_sched_barrier(0);
    long long t3 = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
    if (l == 0) {
        cyc[0] = t1 - t0;
        cyc[1] = t2 - t1;
        cyc[2] = t3 - t2;
    }
    out[256 + l] = x[0] + y[0] + p[0] + q[0] + r2[0] + s2[0];
}
int main() {
    float ha[192], hb[192];
    for (int i = 0; i < 192; ++i) {
        ha[i] = (float)((i * 37 + 11) % 23) - 11.0f;
        hb[i] = (float)((i * 53 + 5) % 19) - 9.0f;
    }
    float *da, *db, *dout;
    long long *dc;
    hipMalloc(&da, sizeof ha);
    hipMalloc(&db, sizeof hb);
    hipMalloc(&dout, 320 * 4);
    hipMalloc(&dc, 3 * 8);
    hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
    hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, 1, 64, 0, 0, da, db, dout, dc);
    float h[320];
    long long c[3];
    hipMemcpy(h, dout, sizeof h, hipMemcpyDeviceToHost);
    hipMemcpy(c, dc, sizeof c, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l) {
        const int bb = l / 4, j = l % 4;
        for (int i = 0; i < 4; ++i) {
            float e = 0;
            for (int s = 0; s < 3; ++s) e += ha[s * 64 + 4 * bb + i] * hb[s * 64 + 4 * bb + j];
            if (e != h[l * 4 + i]) {
                if (bad < 8) printf("lane %d reg %d: got %g want %g\n", l, i, h[l * 4 + i], e);
                bad++;
            }
        }
    }
    printf("4x4x1 layout mismatches: %d of 256\n", bad);
    printf("cycles: 64 dependent 4x4x1 %lld (%.1f each), 64 dependent 16x16x4 %lld (%.1f each), 64 as 4 chains 4x4x1 %lld (%.1f each)\n",
           c[0], c[0] / 64.0, c[1], c[1] / 64.0, c[2], c[2] / 64.0);
    return bad != 0;
}
