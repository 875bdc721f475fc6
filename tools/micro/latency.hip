// Microbenchmark: latency of one round of loads at kernel start, depending on how the data
// was produced by the previous kernel (plain stores from 1 block, fp64 atomics from all blocks,
// or untouched).  hipcc --offload-arch=gfx950 -O3 latency.hip -o latency
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include <algorithm>

__global__ void produce_plain(double *x, int n) {
    if (blockIdx.x == 0) for (int i = threadIdx.x; i < n; i += blockDim.x) x[i] = i * 0.5;
}
__global__ void produce_atomic(double *x, int n, int R) {
    double *d = x + (blockIdx.x % R) * n;
    for (int i = threadIdx.x; i < n; i += blockDim.x) unsafeAtomicAdd(d + i, 1.0);
}
__global__ void consume(const double *x, int n, int nload, unsigned long long *t, double *sink) {
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    double s = 0;
    double v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = x[min((int)(threadIdx.x + k * blockDim.x), n - 1) + 0 * nload];
#pragma unroll
    for (int k = 0; k < 16; ++k) s += (k < nload) ? v[k] : 0.0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { t[blockIdx.x * 2] = t0; t[blockIdx.x * 2 + 1] = t1; }
    if (s == 12345.0) sink[0] = s;
}

int main() {
    const int G = 256, n = 582 * 8;
    double *x, *sink; unsigned long long *t;
    hipMalloc(&x, sizeof(double) * n * 8); hipMalloc(&sink, 8); hipMalloc(&t, sizeof(unsigned long long) * 2 * G);
    hipMemset(x, 0, sizeof(double) * n * 8);
    std::vector<unsigned long long> h(2 * G);
    const char *names[] = {"untouched", "plain-1-block", "atomic-256-blocks"};
    for (int mode = 0; mode < 3; ++mode) {
        for (int rep = 0; rep < 3; ++rep) {
            if (mode == 1) hipLaunchKernelGGL(produce_plain, dim3(G), dim3(512), 0, 0, x, n);
            if (mode == 2) hipLaunchKernelGGL(produce_atomic, dim3(G), dim3(512), 0, 0, x, 582, 8);
            hipLaunchKernelGGL(consume, dim3(G), dim3(512), 0, 0, x, n, 16, t, sink);
            hipDeviceSynchronize();
        }
        hipMemcpy(h.data(), t, sizeof(unsigned long long) * 2 * G, hipMemcpyDeviceToHost);
        std::vector<double> lat(G);
        for (int b = 0; b < G; ++b) lat[b] = (h[2 * b + 1] - h[2 * b]) * 0.01;
        std::sort(lat.begin(), lat.end());
        printf("%-20s load-round latency us: min %.2f med %.2f max %.2f\n", names[mode], lat[0], lat[G / 2], lat[G - 1]);
    }
    return 0;
}
