// Microbenchmark: host-visible round trip of a small launch sequence (the shape of one baseline
// evaluate / one host FVP call), by how the host learns that the work is done:
//   sync    hipStreamSynchronize
//   event   hipEventRecord + hipEventSynchronize
//   spin    the last kernel stores a sequence number into pinned coherent host memory after its data
//           (system-scope release); the host spins on it
//   wrval   hipStreamWriteValue32 of the sequence number after the last kernel (no kernel change); the
//           host spins on it
//   query   hipEventRecord, then the host spins on hipEventQuery
// for 1 and 3 kernels per round trip, on a non-blocking stream.  Also: the host's enqueue cost of
// one launch.   hipcc --offload-arch=gfx950 -O3 host_wait.hip -o host_wait
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <algorithm>
#include <chrono>
#include <vector>

__global__ void work(const double *in, double *out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = in[i] * 1.5 + 1.0;
}
__global__ void finish(const double *in, double *hout, int n, unsigned *hflag, unsigned seq) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) hout[i] = in[i];
    __syncthreads();
    if (threadIdx.x == 0 && hflag) {
        __threadfence_system();
        __hip_atomic_store(hflag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    const int n = 562, reps = 3000;
    hipStream_t st;
    hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    double *a, *b, *h, *hd;
    unsigned *flag, *flag_d;
    hipMalloc(&a, sizeof(double) * n);
    hipMalloc(&b, sizeof(double) * n);
    hipMemset(a, 0, sizeof(double) * n);
    hipHostMalloc((void **)&h, sizeof(double) * n, hipHostMallocMapped | hipHostMallocCoherent);
    hipHostGetDevicePointer((void **)&hd, h, 0);
    hipHostMalloc((void **)&flag, 64, hipHostMallocMapped | hipHostMallocCoherent);
    hipHostGetDevicePointer((void **)&flag_d, flag, 0);
    *flag = 0;
    hipEvent_t ev;
    hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    unsigned seq = 0;
    const char *wname[] = {"sync", "event", "spin", "wrval", "query"};
    for (int kernels : {1, 3})
        for (int how = 0; how < 5; ++how) {
            std::vector<double> t(reps);
            for (int r = 0; r < reps; ++r) {
                const double t0 = now_us();
                ++seq;
                for (int k = 0; k + 1 < kernels; ++k)
                    hipLaunchKernelGGL(work, dim3(3), dim3(256), 0, st, (const double *)a, b, n);
                hipLaunchKernelGGL(finish, dim3(3), dim3(256), 0, st, (const double *)b, hd, n,
                                   how == 2 ? flag_d : nullptr, seq);
                if (how == 0) hipStreamSynchronize(st);
                else if (how == 1) {
                    hipEventRecord(ev, st);
                    hipEventSynchronize(ev);
                } else if (how == 4) {
                    hipEventRecord(ev, st);
                    while (hipEventQuery(ev) == hipErrorNotReady) {}
                } else {
                    if (how == 3 && hipStreamWriteValue32(st, flag_d, seq, 0) != hipSuccess) {
                        printf("hipStreamWriteValue32 failed\n");
                        return 1;
                    }
                    long spins = 0;
                    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq)
                        if (++spins > 2000000000L) { printf("spin bound hit\n"); return 1; }
                }
                t[r] = now_us() - t0;
            }
            hipStreamSynchronize(st);
            std::sort(t.begin(), t.end());
            printf("%d kernel(s) + %-5s: round trip us  p10 %.2f  med %.2f  p90 %.2f\n", kernels, wname[how],
                   t[reps / 10], t[reps / 2], t[reps * 9 / 10]);
        }
    // host enqueue cost of one launch (no wait inside the loop)
    {
        std::vector<double> t(reps);
        for (int r = 0; r < reps; ++r) {
            const double t0 = now_us();
            hipLaunchKernelGGL(work, dim3(3), dim3(256), 0, st, (const double *)a, b, n);
            t[r] = now_us() - t0;
            if (r % 64 == 63) hipStreamSynchronize(st);
        }
        hipStreamSynchronize(st);
        std::sort(t.begin(), t.end());
        printf("enqueue one launch: us  p10 %.2f  med %.2f  p90 %.2f\n", t[reps / 10], t[reps / 2], t[reps * 9 / 10]);
    }
    return 0;
}
