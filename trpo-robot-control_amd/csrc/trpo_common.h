/*
 * trpo_common.h -- definitions shared by the device translation units
 * (trpo_kernels.hip: FVP / CG;  trpo_update.hip: the TRPO_Update path).
 * Internal to libtrpo_mi355x.so; the public ABI is include/trpo_mi355x.h.
 */
#ifndef TRPO_COMMON_H
#define TRPO_COMMON_H

#include <hip/hip_runtime.h>
#include <chrono>
#include <stdio.h>

#include "trpo_dev.h"

#define MAXL 8

enum { ACT_L = 0, ACT_T = 1, ACT_O = 2, ACT_S = 3 };

// Network description in the reference's flat parameter layout
// (src/TRPO_FVP.c:194-215): W[i] row-major [in][out] at woff[i], B[i] at boff[i],
// LogStd[A] at P - A.
struct Net {
    int nl;
    int L[MAXL];
    int act[MAXL];
    int P;
    int woff[MAXL], boff[MAXL];
    int A;
};

#define HCHK(x)                                                                            \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "[trpo_mi355x] HIP error %s at %s:%d\n", hipGetErrorString(e_), \
                    __FILE__, __LINE__);                                                   \
            return -2;                                                                     \
        }                                                                                  \
    } while (0)

// Every device allocation of the library goes through here.  Diagnostics: TRPO_DEBUG_POISON=<byte> fills
// each new allocation with that byte (and waits) before first use, so a kernel that reads device memory
// the library never wrote -- memory a caller's runtime may hand back still holding another allocation's
// bytes -- shows up as a wrong result instead of reading the zeros of fresh pages.
#include <stdlib.h>
static inline hipError_t trpo_malloc(void **p, size_t bytes) {
    const hipError_t e = hipMalloc(p, bytes);
    const char *pz = getenv("TRPO_DEBUG_POISON");
    if (e == hipSuccess && pz && *p) {
        if (hipMemset(*p, atoi(pz) & 0xff, bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
            (void)hipGetLastError();
    }
    return e;
}

// Pinned host staging buffers that the host writes and kernels read (uploads), or kernels write and
// the host reads (results through the mapped pointer), are allocated COHERENT (hipHostMallocDefault is
// non-coherent under HIP_HOST_COHERENT=0, the default: the GPU may cache its lines), and are moved by
// copy kernels through the mapped pointer (~5 us against ~20 us for a pageable hipMemcpyAsync).
// Round 2 blamed hipMemcpyAsync for ranks of the host-group all-reduce diverging in whole 512-element
// slices (6 of 10 sharded 2x64 solves, tools/diag/shard_race.py); round 4 re-ran it with the
// hipMemcpyAsync form restored (TRPO_HGROUP_MEMCPY=1) on top of the cg_axpy same-launch fix: 0 of 10,
// like the copy kernels (profiles/r04_diag/torch_first_bisect_and_probes.log) -- the divergence was
// the cg_axpy race (one 512-element block), not the copy engine.
#define TRPO_HOST_COHERENT (hipHostMallocMapped | hipHostMallocCoherent)

static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// fp64 tanh for the device fp64 paths (precision mode, policy gradient, line search, baseline):
// |x| < 0.55: x + x^3 Q(x^2), Q of degree 9 fitted in extended precision (tools/fit_tanh64.py,
// max relative error 5.4e-16); else 1 - 2 / (e^{2|x|} + 1) (2.7e-16).  ~3x fewer instructions
// than the device libm tanh, which is double-double throughout (it dominated the fp64 surrogate).
__device__ __forceinline__ double tanh64(double x) {
    const double a = fabs(x), u = x * x;
    double q = 6.76744223569079683e-05;
    q = fma(q, u, -2.34387837673838705e-04);
    q = fma(q, u, 5.93821938760988777e-04);
    q = fma(q, u, -1.45812091104440249e-03);
    q = fma(q, u, 3.59269513652666532e-03);
    q = fma(q, u, -8.86331213798425936e-03);
    q = fma(q, u, 2.18694943489975979e-02);
    q = fma(q, u, -5.39682542017260666e-02);
    q = fma(q, u, 1.33333333337541271e-01);
    q = fma(q, u, -3.33333333333355408e-01);
    const double small = fma(a * u, q, a);
    const double big = a > 22.0 ? 1.0 : 1.0 - 2.0 / (exp(2.0 * a) + 1.0);
    return copysign(a < 0.55 ? small : big, x);
}

// Waits until the nf flag words in pinned host memory read seq.  Spinning answers ~4.7 us sooner than
// hipStreamSynchronize for one small launch (tools/micro/host_wait: 6.9 vs 11.6 us round trip); after
// the first query_after_us the stream is queried between spins, so a launch that failed returns its error
// instead of spinning (and one that completed without its flags is an error too).
static inline int trpo_wait_host_flags(hipStream_t st, const unsigned *flags, int nf, unsigned seq, long query_after_us) {
    const auto t0 = std::chrono::steady_clock::now();
    int k = 0;                                   // flags[0 .. k) already read seq
    for (unsigned long i = 1;; ++i) {
        while (k < nf && __atomic_load_n(flags + k, __ATOMIC_ACQUIRE) == seq) ++k;
        if (k == nf) return 0;
        if ((i & 63) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(query_after_us)) {
            const hipError_t e = hipStreamQuery(st);
            if (e == hipSuccess) {
                while (k < nf && __atomic_load_n(flags + k, __ATOMIC_ACQUIRE) == seq) ++k;
                return k == nf ? 0 : -2;
            }
            if (e != hipErrorNotReady) return -2;
        }
        __builtin_ia32_pause();
    }
}

// What the TRPO_Update translation unit may see of a device context.
struct trpo_dev_view {
    int device;
    hipStream_t stream;
    Net net;
    const double *theta64;     // natural theta (W, B, ..., LogStd), fp64
    const double *std64;       // the data file's Std (FVP sigma), fp64 [A]
    const double *obs64;       // local observations [n][L0], fp64
    size_t n;                  // local samples
    double n_total;            // global samples (all ranks)
    double *vec_b;             // CG right-hand side slot (TRPO_VEC_B)
    double *vec_x, *vec_v, *vec_z;
    const int *cg_iter;        // device: iterations of the last CG solve
    const double *cg_hist;     // device: its (rdotr, |x|) history, 2 per iteration
    const double *cg_stats;    // device: its statistics (Ctl::orth, Ctl::alpha[]), TRPO_CG_STATS doubles
};
void trpo_dev_get_view(trpo_dev *d, trpo_dev_view *v);
// in-place fp64 sum over the attached RCCL communicator (no-op without one)
int trpo_dev_allreduce64(trpo_dev *d, double *buf, size_t count);
// policy-gradient weight/bias sums (unnormalised, all ranks) by the MFMA tile kernel in MODE 1;
// roll64 = [n][2A+1] Mean, Action, Adv.  *zacc receives the device vector (P - A entries).
// Returns 1 when the shape has no tile kernel (caller uses the generic fp64 kernel).
// roll_gen: the rollout's upload generation -- its fp32 (Action - Mean) / Adv rows are rebuilt only
// when it changes.
int trpo_dev_pg_sums_fast(trpo_dev *d, const double *roll64, unsigned roll_gen, const double **zacc);
int trpo_dev_pg_prepare(trpo_dev *d, const double *roll64, unsigned roll_gen);
// the update path's CG (graph-replayed unless TRPO_CG_GRAPH=0: it sits between other kernels)
int trpo_dev_cg_in_sequence(trpo_dev *d, size_t maxiter, double resth);
// whether the context has a collective attached (RCCL, host group or peer exchange): its waits are bounded
int trpo_dev_has_collective(const trpo_dev *d);
// forward-cache bookkeeping after a CG solve
void trpo_dev_ycache_written(trpo_dev *d);
// per-context storage of the update path (owned by trpo_update.hip)
void **trpo_dev_update_state(trpo_dev *d);
void trpo_update_state_free(void *state);

// Peer-window exchange (trpo_peer.hip): one-shot all-reduce of small fp64 vectors over xGMI.
#define PEER_WMAX 16                 // ranks
#define PEER_HANDLE_BYTES 64         // one exported window (hipIpcMemHandle_t)
struct trpo_peer;
trpo_peer *trpo_peer_create(int device, size_t slot_doubles);
void trpo_peer_destroy(trpo_peer *p);
int trpo_peer_handle(trpo_peer *p, void *h64);
void *trpo_peer_window(trpo_peer *p);
int trpo_peer_connect(trpo_peer *p, int rank, int world, const void *handles, void *const *local, hipStream_t st);
int trpo_peer_allreduce(trpo_peer *p, hipStream_t st, const double *in, int R, int Rstride, int count, double *out,
                        const int *done);
int trpo_peer_error(const trpo_peer *p);
size_t trpo_peer_slot(const trpo_peer *p);
int trpo_peer_proto(const trpo_peer *p);      // 1 flag form, 3 / 4 tagged granules (4: split roles)
void trpo_peer_report(trpo_peer *p);          // prints a failed exchange's error records once (stderr)
void trpo_peer_set_error(trpo_peer *p);

#endif
