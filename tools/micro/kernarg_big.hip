// Does a kernel take a 4.5 KB by-value argument (the [16,16,16,1] baseline's 561 parameters) on
// gfx950, and what does its launch cost the host against a pointer argument?
//   hipcc --offload-arch=gfx950 -O3 kernarg_big.hip -o kernarg_big
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <algorithm>
#include <chrono>
#include <vector>

struct Theta { double v[561]; };
__global__ void by_value(Theta t, double *out) {
    __shared__ double s[561];
    for (int q = threadIdx.x; q < 561; q += blockDim.x) s[q] = t.v[q];
    __syncthreads();
    if (threadIdx.x == 0) {
        double a = 0;
        for (int q = 0; q < 561; ++q) a += s[q];
        out[blockIdx.x] = a;
    }
}
__global__ void by_ptr(const double *t, double *out) {
    __shared__ double s[561];
    for (int q = threadIdx.x; q < 561; q += blockDim.x) s[q] = t[q];
    __syncthreads();
    if (threadIdx.x == 0) {
        double a = 0;
        for (int q = 0; q < 561; ++q) a += s[q];
        out[blockIdx.x] = a;
    }
}
static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
int main() {
    Theta th;
    double want = 0;
    for (int q = 0; q < 561; ++q) { th.v[q] = 0.25 * q + 1; want += th.v[q]; }
    double *out, *tp;
    if (hipMalloc(&out, 8 * 128) != hipSuccess || hipMalloc(&tp, sizeof th) != hipSuccess) return 2;
    if (hipMemcpy(tp, th.v, sizeof th, hipMemcpyHostToDevice) != hipSuccess) return 2;
    hipStream_t st;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return 2;
    for (int mode = 0; mode < 2; ++mode) {
        const int reps = 3000;
        std::vector<double> t(reps), w(reps);
        for (int r = 0; r < reps; ++r) {
            th.v[0] = 1.0 + r;                                     // a new theta every call
            const double t0 = now_us();
            if (mode == 0) hipLaunchKernelGGL(by_value, dim3(94), dim3(256), 0, st, th, out);
            else hipLaunchKernelGGL(by_ptr, dim3(94), dim3(256), 0, st, (const double *)tp, out);
            const double t1 = now_us();
            if (hipStreamSynchronize(st) != hipSuccess) { printf("launch failed: %s\n", hipGetErrorString(hipGetLastError())); return 1; }
            t[r] = t1 - t0;
            w[r] = now_us() - t0;
            if (mode == 0 && r == reps - 1) {
                double h[94];
                hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost);
                double exp = want - 1.0 + (1.0 + r);
                int bad = 0;
                for (int b = 0; b < 94; ++b) bad += h[b] != exp;
                printf("by-value argument (%zu B): %s\n", sizeof th, bad ? "WRONG" : "ok");
            }
        }
        std::sort(t.begin(), t.end());
        std::sort(w.begin(), w.end());
        printf("%-9s enqueue us med %.2f p90 %.2f | round trip (sync) med %.2f p90 %.2f\n", mode ? "by-ptr" : "by-value",
               t[reps / 2], t[reps * 9 / 10], w[reps / 2], w[reps * 9 / 10]);
    }
    return 0;
}
