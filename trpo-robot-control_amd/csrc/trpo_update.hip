// trpo_update.hip -- gfx950 kernels for the rest of one TRPO policy update
// (reference src/TRPO_Update.c), around the FVP/CG solve of trpo_kernels.hip:
//
//   * policy gradient b = (1/N) sum_n grad_theta [ Adv_n * loglik ]   (:254-378)
//       output seed  G = Adv (Action - Mean) / sigma^2,  sigma = exp(LogStd)
//       LogStd part  Adv ((Action - Mean)^2 / sigma^2 - 1)
//       then ordinary backprop through the policy MLP;
//   * surrogate sums for the backtracking line search               (:951-981)
//       surr_k = sum_n Adv_n exp(0.5 sum_i [tx^2 - tn^2 + log Std_i - LogStd'_i])
//       for candidates theta_k = theta + 2^-k fullstep, several k per launch.
//
// Precision of the policy gradient.  DEFAULT (shapes with an MFMA tile kernel): the weight / bias
// part runs on the fp32 tile kernel in its policy-gradient mode (trpo_dev_pg_sums_fast;
// (Action - Mean) and Adv are rounded to fp32 by pg_prep_kernel, per-sample products in fp32,
// cross-tile sums in fp64) and only the LogStd part and sum(Adv) are fp64 (pg_logstd_kernel);
// measured 1.2e-7 relative to the reference's fp64 gradient (tests allow 2e-6).
// TRPO_UPDATE_GENERIC=1, shapes without a tile kernel, and the fp64 precision mode take the
// generic pg_kernel below: fp64 throughout, reference-exact to ~1e-15.
// The generic kernels (pg_kernel, the line-search surrogate) are written for fidelity first:
// fp64, one sample per lane, 64-sample passes per one-wave workgroup, the pass's activations
// staged in LDS ([row][64], up to 160 KB; a global scratch beyond that), weights read with
// wave-uniform scalar loads.  Cross-sample sums are fixed-order (lane order within a pass, block
// order across blocks), so results are deterministic; multi-GPU ranks add their shard sums with
// one RCCL all-reduce.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "trpo_common.h"

constexpr int UT = 64;                     // samples per pass == threads per workgroup
constexpr int LDS_CAP = 160 * 1024;        // gfx950 LDS per workgroup

struct UpdState {
    double *roll = nullptr;                // [n][2A+1]: Mean[A], Action[A], Adv
    size_t roll_cap = 0, roll_n = 0;
    int have_roll = 0;
    double *ws = nullptr;                  // global activation scratch (big nets only)
    size_t ws_cap = 0;
    double *slabs = nullptr;               // per-block partial sums
    size_t slab_cap = 0;
    double *sum = nullptr;                 // [P + 1]
    double *fs = nullptr;                  // fullstep [P]
    double *sums = nullptr;                // [64]
    double *tpad = nullptr;                // register path: padded parameters [nk][PADW]
    size_t tpad_cap = 0;
    double *tk = nullptr;                  // generic path: the line-search candidates [nk][P]
    size_t tk_cap = 0;
    int lds_set = 0;
    // pinned, device-mapped host buffer: results are written into it by a kernel (no copy-engine
    // round trips through pageable memory); fullstep goes the other way through it
    double *hst = nullptr, *hst_dev = nullptr;
    size_t hst_cap = 0;
    unsigned seq = 0;                       // export_solve_kernel's flags: the last update's sequence number
    size_t flag_at = 0;                     // where they were zeroed last (they move with maxiter)
    unsigned roll_gen = 0;                 // bumped by every rollout upload
};

void trpo_update_state_free(void *state) {
    UpdState *u = (UpdState *)state;
    if (!u) return;
    void *ptrs[] = {u->roll, u->ws, u->slabs, u->sum, u->fs, u->sums, u->tpad, u->tk};
    for (void *p : ptrs)
        if (p) hipFree(p);
    if (u->hst) hipHostFree(u->hst);
    delete u;
}

__device__ __forceinline__ double act_y64(int a, double x) {
    switch (a) {
    case ACT_T: return tanh64(x);
    case ACT_O: return 0.1 * x;
    case ACT_S: return 1.0 / (1.0 + exp(-x));
    default: return x;
    }
}
// d(act)/dx applied to an upstream gradient, expressed through y = act(x)
__device__ __forceinline__ double act_d64(int a, double y, double g) {
    switch (a) {
    case ACT_T: return g * (1.0 - y * y);
    case ACT_O: return 0.1 * g;
    case ACT_S: return g * y * (1.0 - y);
    default: return g;
    }
}

// Plain parameters, or the line-search candidate theta + sf * fullstep (sf = 2^-k, so
// sf * fullstep is exact and the sum rounds once, as xnew[i] = x[i] + stepfrac*fullstep[i]).
struct ThetaPlain {
    const double *__restrict__ t;
    __device__ double operator[](int i) const { return t[i]; }
};
struct ThetaStep {
    const double *__restrict__ t;
    const double *__restrict__ f;
    double sf;
    __device__ double operator[](int i) const { return t[i] + sf * f[i]; }
};

// LDS / scratch activation rows are [row][RS]: the odd stride puts the rows a wave reads at
// the same sample index in different banks during the contraction
constexpr int RS = UT + 1;

// forward pass of sample s into Y rows (rows of layer i start at roff[i]);
// src/TRPO_Update.c:262-293 / :954-976
#ifndef FWD_JB
#define FWD_JB 4            // outputs per sweep over a layer's inputs
#endif
template <class TH>
__device__ void forward64(const Net &net, const TH &th, const double *__restrict__ obs, int s, bool live,
                          double *Y, const int *roff, int tid) {
    const int L0 = net.L[0];
    for (int k = 0; k < L0; ++k) Y[k * RS + tid] = live ? obs[(long)s * L0 + k] : 0.0;
    for (int i = 0; i + 1 < net.nl; ++i) {
        const int in = net.L[i], out = net.L[i + 1], a = net.act[i + 1];
        const int wo = net.woff[i], bo = net.boff[i];
        int j = 0;
        // four outputs per sweep over the inputs: one LDS read of Y feeds four chains (each chain
        // keeps the reference's bias-first, k-ascending order, so the sums are unchanged)
        for (; j + FWD_JB <= out; j += FWD_JB) {
            double x[FWD_JB];
#pragma unroll
            for (int jj = 0; jj < FWD_JB; ++jj) x[jj] = th[bo + j + jj];
#pragma unroll 16
            for (int k = 0; k < in; ++k) {
                const double y = Y[(roff[i] + k) * RS + tid];
                const int w = wo + k * out + j;
#pragma unroll
                for (int jj = 0; jj < FWD_JB; ++jj) x[jj] += y * th[w + jj];
            }
            double *Yo = Y + (roff[i + 1] + j) * RS + tid;
#pragma unroll
            for (int jj = 0; jj < FWD_JB; ++jj) Yo[jj * RS] = act_y64(a, x[jj]);
        }
        for (; j < out; ++j) {
            double x = th[bo + j];
#pragma unroll 4
            for (int k = 0; k < in; ++k) x += Y[(roff[i] + k) * RS + tid] * th[wo + k * out + j];
            Y[(roff[i + 1] + j) * RS + tid] = act_y64(a, x);
        }
    }
}

__device__ __forceinline__ void row_offsets(const Net &net, int *roff) {
    roff[0] = 0;
    for (int i = 0; i < net.nl; ++i) roff[i + 1] = roff[i] + net.L[i];
}

// Sum over the pass's UT samples of every gradient entry, one parameter per thread, added into
// the block's slab (fixed order).  yoff[i]: first row of layer i's outputs y_i (i < nl-1);
// goff[i]: first row of the pre-activation gradient of layer i+1; gl: first of the A GLogStd
// rows, followed by the Adv row (slab index P).
__device__ void contract_pass(const Net &net, const double *Y, const int *yoff, const int *goff, int gl,
                              double *__restrict__ slab, int tid) {
    const int P = net.P, A = net.A;
    for (int q = tid; q <= P; q += UT) {
        const double *u = nullptr, *w = nullptr;
        if (q >= P - A) {
            w = Y + (long)(gl + q - (P - A)) * RS;
        } else {
            int i = 0;
            while (i + 2 < net.nl && q >= net.woff[i + 1]) ++i;
            const int in = net.L[i], out = net.L[i + 1], local = q - net.woff[i];
            if (local < in * out) {
                u = Y + (long)(yoff[i] + local / out) * RS;
                w = Y + (long)(goff[i] + local % out) * RS;
            } else {
                w = Y + (long)(goff[i] + local - in * out) * RS;
            }
        }
        double acc = 0.0;
        if (u) {
#pragma unroll 16
            for (int t = 0; t < UT; ++t) acc += u[t] * w[t];
        } else {
#pragma unroll 16
            for (int t = 0; t < UT; ++t) acc += w[t];
        }
        slab[q] += acc;
    }
}

// Output seed of the policy gradient for one sample (src/TRPO_Update.c:297-303):
// g = Adv (Action - Mean) / sigma^2 and the LogStd term, sigma = exp(LogStd).
__device__ __forceinline__ void pg_seed(const double *rw, int A, int i, double logstd, double adv, double &g,
                                        double &gls) {
    const double es = exp(logstd);
    const double temp = (rw[A + i] - rw[i]) / es;
    g = adv * temp / es;
    gls = adv * (temp * temp - 1.0);
}

// Policy gradient partial sums, any depth / widths: block b accumulates, over its 64-sample
// passes, the unnormalised gradient [GW, GB per layer, GLogStd] (src/TRPO_Update.c:295-378)
// plus sum(Adv) at index P, into slabs[b][P + 1].  Activations in Y rows (LDS or scratch).
template <bool LDSY>
__global__ void __launch_bounds__(UT)
pg_kernel(Net net, const double *__restrict__ th, const double *__restrict__ obs, const double *__restrict__ roll,
          int n, double *ws, int rows, int use_lds, double *__restrict__ slabs) {
    extern __shared__ double lds64[];
    const int tid = threadIdx.x;
    // LDSY (compile time): with a run-time select hipcc cannot tell LDS from global and makes every
    // Y access a flat load / store (one lgkmcnt for LDS and the scalar theta loads alike: round 5)
    double *Y = LDSY ? lds64 : ws + (long)blockIdx.x * rows * RS;
    (void)use_lds;
    int roff[MAXL + 1];
    row_offsets(net, roff);
    const int tot = roff[net.nl], P = net.P, A = net.A, last = net.nl - 1;
    const int G0 = tot, GL = 2 * tot;          // gradient rows mirror Y's; then GLogStd rows + Adv row
    int goff[MAXL];
    for (int i = 0; i + 1 < net.nl; ++i) goff[i] = G0 + roff[i + 1];
    double *slab = slabs + (long)blockIdx.x * (P + 1);
    const ThetaPlain T{th};
    for (int q = tid; q <= P; q += UT) slab[q] = 0.0;
    const int npass = (n + UT - 1) / UT;
    for (int pass = blockIdx.x; pass < npass; pass += gridDim.x) {
        const int s = pass * UT + tid;
        const bool live = s < n;
        forward64(net, T, obs, s, live, Y, roff, tid);
        const double *rw = roll + (long)(live ? s : 0) * (2 * A + 1);
        const double adv = live ? rw[2 * A] : 0.0;
        for (int i = 0; i < A; ++i) {
            double g, gls;
            pg_seed(rw, A, i, th[P - A + i], adv, g, gls);
            Y[(G0 + roff[last] + i) * RS + tid] = live ? g : 0.0;
            Y[(GL + i) * RS + tid] = live ? gls : 0.0;
        }
        Y[(GL + A) * RS + tid] = adv;
        // backprop (src/TRPO_Update.c:305-357); the unused input-layer gradient is skipped
        for (int i = last; i >= 1; --i) {
            const int cur = net.L[i], a = net.act[i];
            for (int j = 0; j < cur; ++j) {
                const int e = (roff[i] + j) * RS + tid;
                Y[G0 * RS + e] = act_d64(a, Y[e], Y[G0 * RS + e]);
            }
            if (i >= 2) {
                const int prev = net.L[i - 1], wo = net.woff[i - 1];
                // FWD_JB outputs per sweep (independent chains, one read of each g_k for all of them;
                // each chain keeps its k-ascending order, so the sums are unchanged: round 5)
                int j = 0;
                for (; j + FWD_JB <= prev; j += FWD_JB) {
                    double t[FWD_JB];
#pragma unroll
                    for (int jj = 0; jj < FWD_JB; ++jj) t[jj] = 0.0;
#pragma unroll 16
                    for (int k = 0; k < cur; ++k) {
                        const double gk = Y[(G0 + roff[i] + k) * RS + tid];
#pragma unroll
                        for (int jj = 0; jj < FWD_JB; ++jj) t[jj] += gk * th[wo + (j + jj) * cur + k];
                    }
#pragma unroll
                    for (int jj = 0; jj < FWD_JB; ++jj) Y[(G0 + roff[i - 1] + j + jj) * RS + tid] = t[jj];
                }
                for (; j < prev; ++j) {
                    double t = 0.0;
#pragma unroll 4
                    for (int k = 0; k < cur; ++k) t += Y[(G0 + roff[i] + k) * RS + tid] * th[wo + j * cur + k];
                    Y[(G0 + roff[i - 1] + j) * RS + tid] = t;
                }
            }
        }
        __syncthreads();
        contract_pass(net, Y, roff, goff, GL, slab, tid);
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Register path: 3 weight layers, every width <= RW.  Each lane keeps its sample's
// activations and gradients in registers (fully unrolled over a zero-padded [RW][RW]
// copy of the weights, read with scalar loads); only the rows the contraction needs go
// through LDS.  Padding adds exact zeros, so the sums equal the unpadded ones.
// ---------------------------------------------------------------------------
constexpr int RW = 16;
constexpr int PADL = RW * RW + RW;               // one padded layer: W [RW][RW] (in, out), B [RW]
constexpr int PADW = 3 * PADL + RW;              // three layers, then LogStd [RW]

// padded parameters theta + sf * fullstep (fs == nullptr: theta itself); blockIdx.y = candidate k
__global__ void pad_theta_kernel(Net net, const double *__restrict__ th, const double *__restrict__ fs, int k0,
                                 double *__restrict__ out) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= PADW) return;
    const double sf = ldexp(1.0, -(k0 + (int)blockIdx.y));
    int m = -1;
    if (e < 3 * PADL) {
        const int i = e / PADL, r = e % PADL;
        const int in = net.L[i], out = net.L[i + 1];
        if (r < RW * RW) {
            const int k = r / RW, j = r % RW;
            if (k < in && j < out) m = net.woff[i] + k * out + j;
        } else if (r - RW * RW < out) {
            m = net.boff[i] + r - RW * RW;
        }
    } else if (e - 3 * PADL < net.A) {
        m = net.P - net.A + e - 3 * PADL;
    }
    out[(long)blockIdx.y * PADW + e] = m < 0 ? 0.0 : (fs ? th[m] + sf * fs[m] : th[m]);
}

__device__ __forceinline__ void act_vec(int a, double (&v)[RW]) {
    if (a == ACT_T) {
#pragma unroll
        for (int j = 0; j < RW; ++j) v[j] = tanh64(v[j]);
    } else if (a == ACT_S) {
#pragma unroll
        for (int j = 0; j < RW; ++j) v[j] = 1.0 / (1.0 + exp(-v[j]));
    } else if (a == ACT_O) {
#pragma unroll
        for (int j = 0; j < RW; ++j) v[j] = 0.1 * v[j];
    }
}
__device__ __forceinline__ void actd_vec(int a, const double (&y)[RW], double (&g)[RW]) {
#pragma unroll
    for (int j = 0; j < RW; ++j) g[j] = act_d64(a, y[j], g[j]);
}
// dst = act(W^T src + B), W [RW][RW] (in, out) -- src/TRPO_Update.c:266-290 order per output
__device__ __forceinline__ void layer_reg(const double *__restrict__ L, int a, const double (&src)[RW],
                                          double (&dst)[RW]) {
#pragma unroll
    for (int j = 0; j < RW; ++j) {
        double x = L[RW * RW + j];
#pragma unroll
        for (int k = 0; k < RW; ++k) x += src[k] * L[k * RW + j];
        dst[j] = x;
    }
    act_vec(a, dst);
}
// dst[k] = sum_j src[j] W[k][j]  (gradient w.r.t. the layer's inputs, :351-356)
__device__ __forceinline__ void back_reg(const double *__restrict__ L, const double (&src)[RW], double (&dst)[RW]) {
#pragma unroll
    for (int k = 0; k < RW; ++k) {
        double t = 0.0;
#pragma unroll
        for (int j = 0; j < RW; ++j) t += src[j] * L[k * RW + j];
        dst[k] = t;
    }
}

__device__ __forceinline__ void forward_reg(const Net &net, const double *__restrict__ tp,
                                            const double *__restrict__ obs, int s, bool live, double (&y0)[RW],
                                            double (&y1)[RW], double (&y2)[RW], double (&y3)[RW]) {
    const int L0 = net.L[0];
#pragma unroll
    for (int k = 0; k < RW; ++k) y0[k] = (live && k < L0) ? obs[(long)s * L0 + k] : 0.0;
    layer_reg(tp, net.act[1], y0, y1);
    layer_reg(tp + PADL, net.act[2], y1, y2);
    layer_reg(tp + 2 * PADL, net.act[3], y2, y3);
}

__device__ __forceinline__ double lld_term(const double *rw, int A, int i, double mean_new, double logstd,
                                           double stdv) {
    const double tx = (rw[A + i] - rw[i]) / stdv;
    const double tn = (rw[A + i] - mean_new) / exp(logstd);
    return tx * tx - tn * tn + log(stdv) - logstd;
}

// the nk line-search candidates theta + 2^-(k0+k) fullstep, k < nk, as [nk][P] (the same
// ThetaStep expression the kernels would otherwise evaluate per weight access, once per element)
__global__ void cand_theta_kernel(const double *__restrict__ th0, const double *__restrict__ fs, int k0, int P,
                                  double *__restrict__ tk) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x, k = blockIdx.y;
    const ThetaStep T{th0, fs, ldexp(1.0, -(k0 + k))};   // pow(0.5, k) exactly
    if (i < P) tk[(long)k * P + i] = T[i];
}

// Line-search surrogate: block (bx, k) sums Adv * exp(LLD) over its passes for candidate k of
// tk (src/TRPO_Update.c:951-981); parts[bx][k].
template <bool LDSY>
__global__ void __launch_bounds__(UT)
surr_kernel(Net net, const double *__restrict__ tk, const double *__restrict__ obs,
            const double *__restrict__ roll, const double *__restrict__ stdv, int n,
            double *ws, int rows, int use_lds, double *__restrict__ parts) {
    extern __shared__ double lds64[];
    const int tid = threadIdx.x, k = blockIdx.y, nk = gridDim.y;
    double *Y = LDSY ? lds64 : ws + ((long)k * gridDim.x + blockIdx.x) * rows * RS;   // see pg_kernel
    (void)use_lds;
    int roff[MAXL + 1];
    row_offsets(net, roff);
    const int P = net.P, A = net.A, last = net.nl - 1;
    const ThetaPlain T{tk + (long)k * P};
    double acc = 0.0;
    const int npass = (n + UT - 1) / UT;
    for (int pass = blockIdx.x; pass < npass; pass += gridDim.x) {
        const int s = pass * UT + tid;
        const bool live = s < n;
        forward64(net, T, obs, s, live, Y, roff, tid);
        if (live) {
            const double *rw = roll + (long)s * (2 * A + 1);
            double lld = 0.0;
            for (int i = 0; i < A; ++i) lld += lld_term(rw, A, i, Y[(roff[last] + i) * RS + tid], T[P - A + i], stdv[i]);
            lld = lld * 0.5;
            acc += exp(lld) * rw[2 * A];
        }
    }
    // fixed-order wave tree
    for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (tid == 0) parts[(long)blockIdx.x * nk + k] = acc;
}

// Line-search surrogate, register path; tp = the nk padded candidates [nk][PADW].
__global__ void __launch_bounds__(UT)
surr_reg_kernel(Net net, const double *__restrict__ tpk, const double *__restrict__ obs,
                const double *__restrict__ roll, const double *__restrict__ stdv, int n,
                double *__restrict__ parts) {
    const int tid = threadIdx.x, k = blockIdx.y, nk = gridDim.y, A = net.A;
    __shared__ double tpw[PADW];
    for (int e = tid; e < PADW; e += UT) tpw[e] = tpk[(long)k * PADW + e];
    __syncthreads();
    double acc = 0.0;
    const int npass = (n + UT - 1) / UT;
    for (int pass = blockIdx.x; pass < npass; pass += gridDim.x) {
        const int s = pass * UT + tid;
        const bool live = s < n;
        int wb = 0;
        asm volatile("" : "+s"(wb));
        const double *tpl = tpw + wb;
        double y0[RW], y1[RW], y2[RW], y3[RW];
        forward_reg(net, tpl, obs, s, live, y0, y1, y2, y3);
        if (live) {
            const double *rw = roll + (long)s * (2 * A + 1);
            double lld = 0.0;
#pragma unroll
            for (int i = 0; i < RW; ++i)
                if (i < A) lld += lld_term(rw, A, i, y3[i], tpl[3 * PADL + i], stdv[i]);
            lld = lld * 0.5;
            acc += exp(lld) * rw[2 * A];
        }
    }
    for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (tid == 0) parts[(long)blockIdx.x * nk + k] = acc;
}

// out[q] = sum_b slabs[b][q] for q < len, in a fixed order (16 strided chains, then in order)
__global__ void __launch_bounds__(256)
sum_slabs64_kernel(const double *__restrict__ slabs, int G, int len, double *__restrict__ out) {
    __shared__ double part[16][17];
    const int tq = threadIdx.x & 15, tj = threadIdx.x >> 4;
    const int q = blockIdx.x * 16 + tq;
    double s = 0.0;
    if (q < len) {
#pragma unroll 8
        for (int b = tj; b < G; b += 16) s += slabs[(long)b * len + q];
    }
    part[tj][tq] = s;
    __syncthreads();
    if (tj == 0 && q < len) {
        double t = 0.0;
        for (int j = 0; j < 16; ++j) t += part[j][tq];
        out[q] = t;
    }
}

// b = sum / N into the CG right-hand side (src/TRPO_Update.c:374-378)
__global__ void pg_finish_kernel(const double *__restrict__ sum, double n_total, int P, double *__restrict__ b) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < P) b[q] = sum[q] / n_total;
}

// same, with the weight/bias sums from the tile kernel (wsum, P - A entries) and the LogStd
// sums (lsum, A entries) kept apart
__global__ void pg_finish2_kernel(const double *__restrict__ wsum, const double *__restrict__ lsum, double n_total,
                                  int P, int A, double *__restrict__ b) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < P) b[q] = (q < P - A ? wsum[q] : lsum[q - (P - A)]) / n_total;
}

// Without a collective (round 6): the LogStd / Adv slab sums and the policy-gradient vector in ONE launch
// instead of sum_slabs64_kernel + pg_finish2_kernel -- blocks [0, nb) write b's weight / bias entries
// (wsum / N), block nb sums the A + 1 LogStd / Adv columns exactly as sum_slabs64_kernel's single block
// does (same partial order, same bits; A + 1 <= 16), keeps them in lsum (sum(Adv) at A) and writes b's
// LogStd entries.
__global__ void pg_sum_finish2_kernel(const double *__restrict__ wsum, const double *__restrict__ slabs, int G, int A,
                                      double n_total, int P, double *__restrict__ lsum, double *__restrict__ b) {
    const int nb = (int)gridDim.x - 1;
    if ((int)blockIdx.x < nb) {
        const int q = blockIdx.x * blockDim.x + threadIdx.x;
        if (q < P - A) b[q] = wsum[q] / n_total;
        return;
    }
    __shared__ double part[16][17];
    const int tq = threadIdx.x & 15, tj = threadIdx.x >> 4, len = A + 1;
    double s = 0.0;
    if (tq < len) {
#pragma unroll 8
        for (int bb = tj; bb < G; bb += 16) s += slabs[(long)bb * len + tq];
    }
    part[tj][tq] = s;
    __syncthreads();
    if (tj == 0 && tq < len) {
        double t = 0.0;
        for (int j = 0; j < 16; ++j) t += part[j][tq];
        lsum[tq] = t;
        if (tq < A) b[P - A + tq] = t / n_total;
    }
}

// LogStd part of the policy gradient and sum(Adv), fp64: block b writes
// slabs[b][i] = sum over its samples of Adv ((Action - Mean)^2 / sigma^2 - 1)  (i < A),
// slabs[b][A] = sum of Adv  (src/TRPO_Update.c:297-303, :372)
__global__ void __launch_bounds__(UT)
pg_logstd_kernel(const double *__restrict__ th, int P, int A, const double *__restrict__ roll, int n,
                 double *__restrict__ slabs) {
    const int tid = threadIdx.x, W = 2 * A + 1;
    const int npass = (n + UT - 1) / UT;
    for (int i = 0; i <= A; ++i) {
        const double es = i < A ? exp(th[P - A + i]) : 1.0;
        double acc = 0.0;
        for (int pass = blockIdx.x; pass < npass; pass += gridDim.x) {
            const int s = pass * UT + tid;
            if (s < n) {
                const double *rw = roll + (long)s * W;
                if (i < A) {
                    const double temp = (rw[A + i] - rw[i]) / es;
                    acc += rw[2 * A] * (temp * temp - 1.0);
                } else {
                    acc += rw[2 * A];
                }
            }
        }
        for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
        if (tid == 0) slabs[(long)blockIdx.x * (A + 1) + i] = acc;
    }
}

// ---------------------------------------------------------------------------
// Line-search surrogate on the fp64 MFMA (v_mfma_f64_16x16x4_f64) for 3-weight-layer policies with
// wide hidden layers (the 2x64 MLPs; src/TRPO_Update.c:951-981).  One wave per 16-sample tile,
// neurons on the MFMA rows and samples on the columns: a layer is acc = B (bias rows) + W^T y, and
// for the fp64 instruction lane (c, g) register r of the accumulator holds neuron g + 4r of sample c
// -- which is exactly the B operand of k-step r of the next layer, so activations never leave the
// registers.  Input neuron of k-step ks (of a 16-wide input tile kt) at lane group g: 16kt + g + 4r,
// r = ks % 4; the candidate's weights are packed in that fragment order (surr_pack_kernel) and
// staged in LDS once per workgroup (lane-contiguous fp64 reads).  Per sample the log-likelihood
// terms of outputs i = g + 4r are gathered to the lane group g = 0 in ascending i, exp(0.5 LLD)
// Adv is accumulated per lane, then the wave tree and the waves in order (fixed-order sums).  The
// dot products round differently from the one-lane-per-sample kernel (MFMA accumulation order);
// the sums agree to ~1e-16 relative.
// ---------------------------------------------------------------------------
static int ensure(double **p, size_t *cap, size_t count, hipStream_t st);
typedef double sd4 __attribute__((ext_vector_type(4)));
constexpr int SM_WAVES = 8;
template <int T0, int T1, int T2>
struct SurrCfg {
    static constexpr int F1 = 0;                             // W1 fragments [T1][4 T0][64]
    static constexpr int F2 = F1 + T1 * 4 * T0 * 64;         // W2 [T2][4 T1][64]
    static constexpr int F3 = F2 + T2 * 4 * T1 * 64;         // W3 [1][4 T2][64]
    static constexpr int B1 = F3 + 4 * T2 * 64;              // biases [16 T1], [16 T2], [16]
    static constexpr int B2 = B1 + 16 * T1;
    static constexpr int B3 = B2 + 16 * T2;
    static constexpr int LS = B3 + 16;                       // LogStd [16]
    static constexpr int LEN = LS + 16;
};

// natural parameter index of pack element e (-1: zero padding)
template <int T0, int T1, int T2>
__device__ int surr_pack_map(const Net &net, int e) {
    using C = SurrCfg<T0, T1, T2>;
    int lo, nks, layer;
    if (e < C::F2) {
        lo = C::F1, nks = 4 * T0, layer = 0;
    } else if (e < C::F3) {
        lo = C::F2, nks = 4 * T1, layer = 1;
    } else if (e < C::B1) {
        lo = C::F3, nks = 4 * T2, layer = 2;
    } else {
        const int A = net.A;
        if (e < C::B2) return e - C::B1 < net.L[1] ? net.boff[0] + e - C::B1 : -1;
        if (e < C::B3) return e - C::B2 < net.L[2] ? net.boff[1] + e - C::B2 : -1;
        if (e < C::LS) return e - C::B3 < A ? net.boff[2] + e - C::B3 : -1;
        return e - C::LS < A ? net.P - A + e - C::LS : -1;
    }
    const int local = e - lo, lane = local & 63, frag = local >> 6;
    const int ot = frag / nks, ks = frag % nks, c = lane & 15, g = lane >> 4;
    const int in = 16 * (ks >> 2) + g + 4 * (ks & 3), out = 16 * ot + c;
    const int L_in = net.L[layer], L_out = net.L[layer + 1];
    return (in < L_in && out < L_out) ? net.woff[layer] + in * L_out + out : -1;
}

// the nk candidates theta + 2^-(k0+k) fullstep in fragment order, [nk][LEN] (fs == nullptr: theta)
template <int T0, int T1, int T2>
__global__ void surr_pack_kernel(Net net, const double *__restrict__ th, const double *__restrict__ fs, int k0,
                                 double *__restrict__ out) {
    using C = SurrCfg<T0, T1, T2>;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= C::LEN) return;
    const int m = surr_pack_map<T0, T1, T2>(net, e);
    const ThetaStep T{th, fs, ldexp(1.0, -(k0 + (int)blockIdx.y))};
    out[(long)blockIdx.y * C::LEN + e] = m < 0 ? 0.0 : (fs ? T[m] : th[m]);
}

__device__ __forceinline__ sd4 act4_64(int a, sd4 x) {
    sd4 y;
#pragma unroll
    for (int r = 0; r < 4; ++r) y[r] = act_y64(a, x[r]);
    return y;
}

template <int T0, int T1, int T2>
__global__ void __launch_bounds__(64 * SM_WAVES)
surr_mfma_kernel(Net net, const double *__restrict__ pk, const double *__restrict__ obs,
                 const double *__restrict__ roll, const double *__restrict__ stdv, int n,
                 double *__restrict__ parts) {
    using C = SurrCfg<T0, T1, T2>;
    __shared__ __attribute__((aligned(16))) double spl[C::LEN];
    __shared__ double wsum[SM_WAVES];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, c = lane & 15, g = lane >> 4;
    const int k = blockIdx.y, nk = gridDim.y;
    static_assert(C::LEN % 2 == 0, "pack length");
    {
        const double2 *src = reinterpret_cast<const double2 *>(pk + (long)k * C::LEN);
        double2 *dst = reinterpret_cast<double2 *>(spl);
        for (int e = tid; e < C::LEN / 2; e += 64 * SM_WAVES) dst[e] = src[e];
    }
    __syncthreads();
    const int L0 = net.L[0], A = net.A, W = 2 * A + 1;
    const int a1 = net.act[1], a2 = net.act[2], a3 = net.act[3];
    const int ntiles = (n + 15) / 16, nwaves = gridDim.x * SM_WAVES;
    double acc = 0.0;
    for (int tile = blockIdx.x * SM_WAVES + wave; tile < ntiles; tile += nwaves) {
        const int s = tile * 16 + c;
        const bool live = s < n;
        const long sc = live ? s : 0;
        // an opaque base per trip: keeps the compiler from hoisting all the (loop-invariant) weight
        // fragment reads out of the loop into ~200 registers
        int wb = 0;
        asm volatile("" : "+v"(wb));
        const double *sp = spl + wb;
        double x0[4 * T0];
#pragma unroll
        for (int ks = 0; ks < 4 * T0; ++ks) {
            const int in = 16 * (ks >> 2) + g + 4 * (ks & 3);
            x0[ks] = (live && in < L0) ? obs[sc * L0 + in] : 0.0;
        }
        sd4 y1[T1], y2[T2];
#pragma unroll
        for (int ot = 0; ot < T1; ++ot) {
            sd4 a;
#pragma unroll
            for (int r = 0; r < 4; ++r) a[r] = sp[C::B1 + 16 * ot + g + 4 * r];
#pragma unroll
            for (int ks = 0; ks < 4 * T0; ++ks)
                a = __builtin_amdgcn_mfma_f64_16x16x4f64(sp[C::F1 + (ot * 4 * T0 + ks) * 64 + lane], x0[ks], a, 0, 0, 0);
            y1[ot] = act4_64(a1, a);
        }
#pragma unroll
        for (int ot = 0; ot < T2; ++ot) {
            sd4 a;
#pragma unroll
            for (int r = 0; r < 4; ++r) a[r] = sp[C::B2 + 16 * ot + g + 4 * r];
#pragma unroll
            for (int kt = 0; kt < T1; ++kt)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    a = __builtin_amdgcn_mfma_f64_16x16x4f64(sp[C::F2 + (ot * 4 * T1 + 4 * kt + r) * 64 + lane],
                                                             y1[kt][r], a, 0, 0, 0);
            y2[ot] = act4_64(a2, a);
        }
        sd4 m;
#pragma unroll
        for (int r = 0; r < 4; ++r) m[r] = sp[C::B3 + g + 4 * r];
#pragma unroll
        for (int kt = 0; kt < T2; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                m = __builtin_amdgcn_mfma_f64_16x16x4f64(sp[C::F3 + (4 * kt + r) * 64 + lane], y2[kt][r], m, 0, 0, 0);
        m = act4_64(a3, m);
        // log-likelihood terms of outputs i = g + 4r (src/TRPO_Update.c:956-976), summed in ascending i
        const double *rw = roll + sc * W;
        double term[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = g + 4 * r;
            term[r] = (live && i < A) ? lld_term(rw, A, i, m[r], sp[C::LS + i], stdv[i]) : 0.0;
        }
        double lld = 0.0;
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int gg = 0; gg < 4; ++gg)
                if (gg + 4 * r < A) lld += __shfl(term[r], c + 16 * gg, 64);
        lld = lld * 0.5;
        if (g == 0 && live) acc += exp(lld) * rw[2 * A];
    }
    for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (lane == 0) wsum[wave] = acc;
    __syncthreads();
    if (tid == 0) {
        double t = 0.0;
        for (int w = 0; w < SM_WAVES; ++w) t += wsum[w];
        parts[(long)blockIdx.x * nk + k] = t;
    }
}

// the MFMA surrogate's shape: 3 weight layers, inputs <= 32, hidden widths <= 64 with equal tile
// counts (16-wide tiles), <= 16 outputs; returns the instantiation index or -1
// (TRPO_SURR_GENERIC=1: the one-lane kernels -- the register kernel for widths <= 16)
static int surr_mfma_shape(const Net &net) {
    const char *e = getenv("TRPO_SURR_GENERIC");
    if (e && atoi(e)) return -1;
    if (net.nl != 4 || net.L[0] > 32 || net.L[3] > 16 || net.L[1] > 64 || net.L[2] > 64) return -1;
    const int T0 = cdiv(net.L[0], 16), T1 = cdiv(net.L[1], 16), T2 = cdiv(net.L[2], 16);
    if (T1 != T2) return -1;
    return (T0 - 1) * 4 + (T1 - 1);      // T0 in {1, 2}, T1 = T2 in {1, 2, 3, 4}
}

template <int T0, int T1>
static int launch_surr_mfma(const Net &net, const double *th, const double *fs, int k0, int nk, double **pk,
                            size_t *pk_cap, const double *obs, const double *roll, const double *stdv, int n, int G,
                            double *parts, hipStream_t st) {
    using C = SurrCfg<T0, T1, T1>;
    if (ensure(pk, pk_cap, (size_t)C::LEN * nk, st)) return -2;
    hipLaunchKernelGGL((surr_pack_kernel<T0, T1, T1>), dim3(cdiv(C::LEN, 256), nk), dim3(256), 0, st, net, th, fs, k0,
                       *pk);
    hipLaunchKernelGGL((surr_mfma_kernel<T0, T1, T1>), dim3(G, nk), dim3(64 * SM_WAVES), 0, st, net,
                       (const double *)*pk, obs, roll, stdv, n, parts);
    HCHK(hipGetLastError());
    return 0;
}

// ---------------------------------------------------------------------------
// device-layer entry points (trpo_dev.h)
// ---------------------------------------------------------------------------
static UpdState *state(trpo_dev *d) {
    void **slot = trpo_dev_update_state(d);
    if (!*slot) *slot = new UpdState();
    return (UpdState *)*slot;
}

static int ensure(double **p, size_t *cap, size_t count, hipStream_t st) {
    if (count <= *cap && *p) return 0;
    if (*p) hipFree(*p);
    *p = nullptr;
    *cap = 0;
    HCHK(trpo_malloc((void **)p, sizeof(double) * (count ? count : 1)));
    HCHK(hipMemsetAsync(*p, 0, sizeof(double) * (count ? count : 1), st));
    *cap = count;
    return 0;
}

static int ensure_host(UpdState *u, size_t count) {
    if (count <= u->hst_cap && u->hst) return 0;
    if (u->hst) hipHostFree(u->hst);
    u->hst = u->hst_dev = nullptr;
    u->hst_cap = 0;
    HCHK(hipHostMalloc((void **)&u->hst, sizeof(double) * count, TRPO_HOST_COHERENT));
    HCHK(hipHostGetDevicePointer((void **)&u->hst_dev, u->hst, 0));
    u->hst_cap = count;
    memset(u->hst, 0, sizeof(double) * count);     // export_solve_kernel's flag words start below any seq
    return 0;
}

// b, x, z (P each), sum(Adv), the CG iteration count and 2 (H) history values -> mapped host memory
// The update's results into the pinned host buffer: b, x, z, the advantage sum, the iteration count, the
// (rdotr, |x|) history and the CG statistics (out + 3P + 5 + H); then every block stores the call's
// sequence number into its own flag word behind its drained system-scope stores, and the host spins on
// the flags instead of a stream sync (round 6, as the baseline evaluate: ~4.7 us sooner per update, one
// launch fewer than a separate statistics copy).
__global__ void export_solve_kernel(const double *__restrict__ b, const double *__restrict__ x,
                                    const double *__restrict__ z, const double *__restrict__ adv,
                                    const int *__restrict__ iter, const double *__restrict__ hist, int P, int H,
                                    const double *__restrict__ stats, double *out, unsigned *flags, unsigned seq) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    constexpr int MS = __HIP_MEMORY_SCOPE_SYSTEM;
    if (i < P) {
        __hip_atomic_store(out + i, b[i], __ATOMIC_RELAXED, MS);
        __hip_atomic_store(out + P + i, x[i], __ATOMIC_RELAXED, MS);
        __hip_atomic_store(out + 2 * P + i, z[i], __ATOMIC_RELAXED, MS);
    }
    if (i == 0) {
        __hip_atomic_store(out + 3 * P, *adv, __ATOMIC_RELAXED, MS);
        __hip_atomic_store(out + 3 * P + 1, (double)*iter, __ATOMIC_RELAXED, MS);
    }
    if (i < H) __hip_atomic_store(out + 3 * P + 2 + i, hist[i], __ATOMIC_RELAXED, MS);
    if (i < TRPO_CG_STATS) __hip_atomic_store(out + 3 * P + 5 + H + i, stats[i], __ATOMIC_RELAXED, MS);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flags + blockIdx.x, seq, __ATOMIC_RELAXED, MS);
}

// Step size of the update (src/TRPO_Update.c:836-846): shs = 0.5 x.Fx, lm = sqrt(shs / max_kl),
// fullstep = x / lm.  One 1024-thread workgroup: strided per-thread partial sums, then the wave tree
// and the waves in order (a fixed order, so every call gives the same bits); shs and lm go to the
// host with the solve's results and the host uses them as they are, so its fullstep x[i] / lm is the
// device's bit for bit (the first line-search candidate is evaluated on the device with it).  The
// summation order is NOT the reference's sequential x.Fx (src/TRPO_Update.c:836-846), so shs differs
// from it by rounding only (relative ~1e-16 of a positive sum); the update goldens' 1e-4 bound on the
// step (tests/test_gpu_update.py) and the printed shs / lagrange lines cover it.
constexpr int STEP_T = 1024;
__global__ void __launch_bounds__(STEP_T)
step_kernel(const double *__restrict__ x, const double *__restrict__ z, int P, double max_kl,
            double *__restrict__ fs, double *__restrict__ shs_lm) {
    __shared__ double wpart[STEP_T / 64];
    __shared__ double lm_s;
    const int tid = threadIdx.x;
    double acc = 0.0;
    for (int i = tid; i < P; i += STEP_T) acc += z[i] * x[i];
    for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if ((tid & 63) == 0) wpart[tid >> 6] = acc;
    __syncthreads();
    if (tid == 0) {
        double t = 0.0;
        for (int w = 0; w < STEP_T / 64; ++w) t += wpart[w];
        const double shs = t * 0.5, lm = sqrt(shs / max_kl);
        lm_s = lm;
        shs_lm[0] = shs;
        shs_lm[1] = lm;
    }
    __syncthreads();
    for (int i = tid; i < P; i += STEP_T) fs[i] = x[i] / lm_s;
}

// small vector copies to / from the mapped host buffer by a kernel (no copy-engine latency)
__global__ void copy64_kernel(const double *__restrict__ src, double *__restrict__ dst, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[i];
}

static int rows_for(const Net &net, bool grads) {
    int tot = 0;
    for (int i = 0; i < net.nl; ++i) tot += net.L[i];
    return grads ? 2 * tot + net.A + 1 : tot;
}

// register path: 3 weight layers, all widths <= RW (env TRPO_UPDATE_GENERIC=1 forces the other)
static bool reg_path(const Net &net) {
    const char *e = getenv("TRPO_UPDATE_GENERIC");
    if (e && atoi(e)) return false;
    if (net.nl != 4) return false;
    for (int i = 0; i < 4; ++i)
        if (net.L[i] > RW) return false;
    return true;
}

static int set_lds_attrs(UpdState *u) {
    if (u->lds_set) return 0;
    HCHK(hipFuncSetAttribute((const void *)pg_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_CAP));
    HCHK(hipFuncSetAttribute((const void *)surr_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_CAP));
    u->lds_set = 1;
    return 0;
}

// activation storage for `blocks` workgroups of `rows` rows: LDS when it fits (returns the
// dynamic LDS bytes), else a global scratch (returns 0)
static int act_storage(UpdState *u, int rows, long blocks, hipStream_t st, int *use_lds) {
    const size_t bytes = sizeof(double) * (size_t)rows * RS;
    if (set_lds_attrs(u)) return -1;
    if (bytes <= (size_t)LDS_CAP) {
        *use_lds = 1;
        return (int)bytes;
    }
    *use_lds = 0;
    if (ensure(&u->ws, &u->ws_cap, (size_t)rows * RS * blocks, st)) return -1;
    return 0;
}

extern "C" int trpo_dev_set_rollout(trpo_dev *d, const double *mean, const double *action, const double *adv,
                                    size_t n) {
    if (!d || (n && (!mean || !action || !adv))) return -1;
    trpo_dev_view v;
    trpo_dev_get_view(d, &v);
    if (n != v.n) return -1;
    HCHK(hipSetDevice(v.device));
    UpdState *u = state(d);
    const int A = v.net.A, W = 2 * A + 1;
    double *h = (double *)malloc(sizeof(double) * (n * W + 1));
    if (!h) return -1;
    for (size_t s = 0; s < n; ++s) {
        memcpy(h + s * W, mean + s * A, sizeof(double) * A);
        memcpy(h + s * W + A, action + s * A, sizeof(double) * A);
        h[s * W + 2 * A] = adv[s];
    }
    int rc = ensure(&u->roll, &u->roll_cap, n * W, v.stream);
    if (!rc && n) rc = hipMemcpyAsync(u->roll, h, sizeof(double) * n * W, hipMemcpyHostToDevice, v.stream) ? -2 : 0;
    if (!rc) rc = trpo_dev_wait_done(d);
    free(h);
    if (rc) return rc;
    u->roll_n = n;
    u->have_roll = 1;
    ++u->roll_gen;
    return 0;
}

// the uploaded rollout back to the host (a twin context's rebuild): mean [n][A], action [n][A], adv [n]
extern "C" int trpo_dev_get_rollout(trpo_dev *d, double *mean, double *action, double *adv) {
    if (!d) return -1;
    trpo_dev_view v;
    trpo_dev_get_view(d, &v);
    UpdState *u = state(d);
    if (!u->have_roll || u->roll_n != v.n) return -3;
    if (!v.n) return 0;
    if (!mean || !action || !adv) return -1;
    HCHK(hipSetDevice(v.device));
    const int A = v.net.A, W = 2 * A + 1;
    double *h = (double *)malloc(sizeof(double) * v.n * W);
    if (!h) return -3;
    int rc = hipMemcpyAsync(h, u->roll, sizeof(double) * v.n * W, hipMemcpyDeviceToHost, v.stream) ? -2 : 0;
    if (!rc) rc = trpo_dev_wait_done(d);
    if (!rc)
        for (size_t s = 0; s < v.n; ++s) {
            memcpy(mean + s * A, h + s * W, sizeof(double) * A);
            memcpy(action + s * A, h + s * W + A, sizeof(double) * A);
            adv[s] = h[s * W + 2 * A];
        }
    free(h);
    return rc;
}

// enqueue the policy gradient into slot B; *adv_dev = device address of the global sum(Adv)
static int enqueue_policy_gradient(trpo_dev *d, const double **adv_dev) {
    if (!d) return -1;
    trpo_dev_view v;
    trpo_dev_get_view(d, &v);
    UpdState *u = state(d);
    if (!u->have_roll || u->roll_n != v.n) return -3;       // rollout missing / stale for this obs
    HCHK(hipSetDevice(v.device));
    const Net &net = v.net;
    const int P = net.P, n = (int)v.n;
    const int G = n ? (cdiv(n, UT) < 1024 ? cdiv(n, UT) : 1024) : 1;
    if (ensure(&u->slabs, &u->slab_cap, (size_t)G * (P + 1), v.stream)) return -2;
    if (!u->sum) HCHK(trpo_malloc((void **)&u->sum, sizeof(double) * (P + 1)));
    const char *eg = getenv("TRPO_UPDATE_GENERIC");
    const double *wsum = nullptr;
    int fast = (eg && atoi(eg)) ? 1 : trpo_dev_pg_sums_fast(d, u->roll, u->roll_gen, &wsum);
    if (fast < 0) return fast;
    if (fast == 0) {
        // weights / biases by the MFMA tile kernel (fp32 per sample, fp64 sums); LogStd + Adv in fp64
        const int A = net.A;
        hipLaunchKernelGGL(pg_logstd_kernel, dim3(G), dim3(UT), 0, v.stream, v.theta64, P, A, u->roll, n, u->slabs);
        if (A + 1 <= 16 && !trpo_dev_has_collective(d)) {
            hipLaunchKernelGGL(pg_sum_finish2_kernel, dim3(cdiv(P - A, 256) + 1), dim3(256), 0, v.stream, wsum,
                               (const double *)u->slabs, G, A, v.n_total, P, u->sum, v.vec_b);
            HCHK(hipGetLastError());
            *adv_dev = u->sum + A;
            return 0;
        }
        hipLaunchKernelGGL(sum_slabs64_kernel, dim3(cdiv(A + 1, 16)), dim3(256), 0, v.stream, u->slabs, G, A + 1,
                           u->sum);
        HCHK(hipGetLastError());
        if (trpo_dev_allreduce64(d, u->sum, (size_t)A + 1)) return -4;
        hipLaunchKernelGGL(pg_finish2_kernel, dim3(cdiv(P, 256)), dim3(256), 0, v.stream, wsum, u->sum, v.n_total,
                           P, A, v.vec_b);
        HCHK(hipGetLastError());
        *adv_dev = u->sum + A;
        return 0;
    }
    {
        const int rows = rows_for(net, true);
        int use_lds = 0;
        const int lds = act_storage(u, rows, G, v.stream, &use_lds);
        if (lds < 0) return -2;
        hipLaunchKernelGGL(use_lds ? pg_kernel<true> : pg_kernel<false>, dim3(G), dim3(UT), lds, v.stream, net,
                           v.theta64, v.obs64, u->roll, n, u->ws, rows, use_lds, u->slabs);
    }
    hipLaunchKernelGGL(sum_slabs64_kernel, dim3(cdiv(P + 1, 16)), dim3(256), 0, v.stream, u->slabs, G, P + 1, u->sum);
    HCHK(hipGetLastError());
    if (trpo_dev_allreduce64(d, u->sum, (size_t)P + 1)) return -4;
    hipLaunchKernelGGL(pg_finish_kernel, dim3(cdiv(P, 256)), dim3(256), 0, v.stream, u->sum, v.n_total, P, v.vec_b);
    HCHK(hipGetLastError());
    *adv_dev = u->sum + P;
    return 0;
}

extern "C" int trpo_dev_policy_gradient(trpo_dev *d, double *b_host, double *adv_sum) {
    const double *adv_dev = nullptr;
    int rc = enqueue_policy_gradient(d, &adv_dev);
    if (rc) return rc;
    trpo_dev_view v;
    trpo_dev_get_view(d, &v);
    if (b_host) HCHK(hipMemcpyAsync(b_host, v.vec_b, sizeof(double) * v.net.P, hipMemcpyDeviceToHost, v.stream));
    if (adv_sum) HCHK(hipMemcpyAsync(adv_sum, adv_dev, sizeof(double), hipMemcpyDeviceToHost, v.stream));
    DSYNC(d);
    return 0;
}

static int enqueue_surrogate(trpo_dev *d, const double *fs, int k0, int nk, double *host_out = nullptr);
// export_solve_kernel's grid and the offset of its flag words in the update's pinned buffer
static int export_blocks(int P, int H) {
    const int m = P > H ? P : H;
    return cdiv(m > TRPO_CG_STATS ? m : TRPO_CG_STATS, 256);
}
static size_t export_flags_at(int P, int H) { return (size_t)3 * P + 5 + H + TRPO_CG_STATS; }

// policy gradient -> B, CG -> X, FVP(x) -> Z, [step + full-step surrogate], results -> mapped host memory
static int enqueue_update_device(trpo_dev *d, size_t maxiter, double resth, double max_kl, bool surr) {
    const double *adv_dev = nullptr;
    int rc = enqueue_policy_gradient(d, &adv_dev);             // :254-378
    if (!rc) rc = trpo_dev_cg_in_sequence(d, maxiter, resth);   // :383-628 (the context's CG graph)
    if (rc) return rc;
    trpo_dev_ycache_written(d);
    trpo_dev_view v;
    trpo_dev_get_view(d, &v);
    rc = trpo_dev_fvp_src(d, v.vec_x);                          // :633-832, z = F x (x read in place)
    if (rc) return rc;
    UpdState *u = state(d);
    const int P = v.net.P, H = 2 * ((int)maxiter + 1);
    // the step size (-> mapped host buffer) and, with surr, the full-step surrogate (the usual outcome
    // of the line search) in the same submission: no host round trip before the first candidate
    hipLaunchKernelGGL(step_kernel, dim3(1), dim3(STEP_T), 0, v.stream, (const double *)v.vec_x,
                       (const double *)v.vec_z, P, max_kl, u->fs, u->hst_dev + 3 * P + 3 + H);
    if (surr) {
        rc = enqueue_surrogate(d, u->fs, 0, 1, u->hst_dev + 3 * P + 2 + H);
        if (rc) return rc;
    }
    if (++u->seq == 0) u->seq = 1;
    if (export_flags_at(P, H) != u->flag_at) {     // a new layout: no stale word may read as this seq
        memset(u->hst + export_flags_at(P, H), 0, sizeof(double) * cdiv(export_blocks(P, H), 2));
        u->flag_at = export_flags_at(P, H);
    }
    hipLaunchKernelGGL(export_solve_kernel, dim3(export_blocks(P, H)), dim3(256), 0, v.stream, v.vec_b, v.vec_x,
                       v.vec_z, adv_dev, v.cg_iter, v.cg_hist, P, H, v.cg_stats, u->hst_dev,
                       (unsigned *)(u->hst_dev + export_flags_at(P, H)), u->seq);
    HCHK(hipGetLastError());
    return 0;
}

extern "C" int trpo_dev_update_solve(trpo_dev *d, size_t maxiter, double resth, double *b, double *x, double *z,
                                     double *adv_sum, size_t *iters, double *rdotr_hist, double *xnorm_hist,
                                     double max_kl, double *surr0, double *shs_lm, double *stats) {
    if (!d || !b || !x || !z || !adv_sum || maxiter > 100000) return -1;
    trpo_dev_view v;
    trpo_dev_get_view(d, &v);
    UpdState *u = state(d);
    if (!u->have_roll || u->roll_n != v.n) return -3;
    HCHK(hipSetDevice(v.device));
    const int P = v.net.P, H = 2 * ((int)maxiter + 1);
    const size_t bytes = sizeof(double) * P;
    const bool surr = surr0 != nullptr;
    // outside any graph: buffers, and the rollout rows of the policy-gradient kernel (new rollout only)
    if (ensure_host(u, export_flags_at(P, H) + cdiv(export_blocks(P, H), 2))) return -2;
    if (!u->fs) HCHK(trpo_malloc((void **)&u->fs, sizeof(double) * P));
    if (trpo_dev_pg_prepare(d, u->roll, u->roll_gen) < 0) return -2;
    // (capturing this whole sequence into one graph was measured: ~3 % faster per update, ~10 ms to
    // capture -- not kept)
    int rc = enqueue_update_device(d, maxiter, resth, max_kl, surr);
    if (rc) return rc;
    if (trpo_dev_has_collective(d)) {
        DSYNC(d);                               // bounded wait, and the collective's own error
    } else if (const int wrc = trpo_wait_host_flags(v.stream, (const unsigned *)(u->hst + export_flags_at(P, H)),
                                               export_blocks(P, H), u->seq, 2000)) {
        return wrc;
    }
    if (surr0) *surr0 = u->hst[3 * P + 2 + H];
    if (stats) memcpy(stats, u->hst + 3 * P + 5 + H, sizeof(double) * TRPO_CG_STATS);
    if (shs_lm) {
        shs_lm[0] = u->hst[3 * P + 3 + H];
        shs_lm[1] = u->hst[3 * P + 4 + H];
    }
    const double *h = u->hst;
    memcpy(b, h, bytes);
    memcpy(x, h + P, bytes);
    memcpy(z, h + 2 * P, bytes);
    *adv_sum = h[3 * P];
    const size_t it = (size_t)h[3 * P + 1];
    if (iters) *iters = it;
    for (size_t i = 0; i <= it && i <= maxiter; ++i) {
        if (rdotr_hist) rdotr_hist[i] = h[3 * P + 2 + 2 * i];
        if (xnorm_hist) xnorm_hist[i] = h[3 * P + 3 + 2 * i];
    }
    return 0;
}

// enqueue the surrogate sums of candidates theta + 2^-k fs, k = k0 .. k0+nk-1 (fs on the device),
// all-reduced over the ranks, into u->sums[0 .. nk)
// host_out (pinned, device-mapped; optional): without a collective the sums are stored there directly
static int enqueue_surrogate(trpo_dev *d, const double *fs, int k0, int nk, double *host_out) {
    trpo_dev_view v;
    trpo_dev_get_view(d, &v);
    UpdState *u = state(d);
    if (!u->have_roll || u->roll_n != v.n) return -3;
    const Net &net = v.net;
    const int n = (int)v.n;
    const int cap = 2048 / nk > 0 ? 2048 / nk : 1;
    const int Gs = n ? (cdiv(n, UT) < cap ? cdiv(n, UT) : cap) : 1;
    if (ensure(&u->slabs, &u->slab_cap, (size_t)Gs * nk, v.stream)) return -2;
    if (!u->sums) HCHK(trpo_malloc((void **)&u->sums, sizeof(double) * 64));
    const int ms = surr_mfma_shape(net);
    if (ms >= 0) {
        // one wave per 16-sample tile, SM_WAVES per workgroup
        const int cap2 = 512 / nk > 0 ? 512 / nk : 1, Gm = n ? (cdiv(cdiv(n, 16), SM_WAVES) < cap2 ? cdiv(cdiv(n, 16), SM_WAVES) : cap2) : 1;
        if (ensure(&u->slabs, &u->slab_cap, (size_t)Gm * nk, v.stream)) return -2;
        int rc = 0;
#define SURR_CASE(i, a, b)                                                                                    \
    case i: rc = launch_surr_mfma<a, b>(net, v.theta64, fs, k0, nk, &u->tpad, &u->tpad_cap, v.obs64, u->roll,    \
                                        v.std64, n, Gm, u->slabs, v.stream);                                      \
        break;
        switch (ms) {
            SURR_CASE(0, 1, 1) SURR_CASE(1, 1, 2) SURR_CASE(2, 1, 3) SURR_CASE(3, 1, 4)
            SURR_CASE(4, 2, 1) SURR_CASE(5, 2, 2) SURR_CASE(6, 2, 3) SURR_CASE(7, 2, 4)
        default: return -1;
        }
#undef SURR_CASE
        if (rc) return rc;
        if (host_out && !trpo_dev_has_collective(d)) {
            hipLaunchKernelGGL(sum_slabs64_kernel, dim3(cdiv(nk, 16)), dim3(256), 0, v.stream, u->slabs, Gm, nk,
                               host_out);
            HCHK(hipGetLastError());
            return 0;
        }
        hipLaunchKernelGGL(sum_slabs64_kernel, dim3(cdiv(nk, 16)), dim3(256), 0, v.stream, u->slabs, Gm, nk, u->sums);
        HCHK(hipGetLastError());
        if (trpo_dev_allreduce64(d, u->sums, (size_t)nk)) return -4;
        if (host_out)
            hipLaunchKernelGGL(copy64_kernel, dim3(1), dim3(64), 0, v.stream, (const double *)u->sums, host_out, nk);
        return 0;
    }
    if (reg_path(net)) {
        if (ensure(&u->tpad, &u->tpad_cap, (size_t)PADW * nk, v.stream)) return -2;
        hipLaunchKernelGGL(pad_theta_kernel, dim3(cdiv(PADW, 256), nk), dim3(256), 0, v.stream, net, v.theta64, fs, k0,
                           u->tpad);
        hipLaunchKernelGGL(surr_reg_kernel, dim3(Gs, nk), dim3(UT), 0, v.stream, net, (const double *)u->tpad,
                           v.obs64, u->roll, v.std64, n, u->slabs);
    } else {
        if (ensure(&u->tk, &u->tk_cap, (size_t)net.P * nk, v.stream)) return -2;
        hipLaunchKernelGGL(cand_theta_kernel, dim3(cdiv(net.P, 256), nk), dim3(256), 0, v.stream, v.theta64, fs, k0,
                           net.P, u->tk);
        const int rows = rows_for(net, false);
        int use_lds = 0;
        const int lds = act_storage(u, rows, (long)Gs * nk, v.stream, &use_lds);
        if (lds < 0) return -2;
        hipLaunchKernelGGL(use_lds ? surr_kernel<true> : surr_kernel<false>, dim3(Gs, nk), dim3(UT), lds, v.stream,
                           net, (const double *)u->tk, v.obs64, u->roll, v.std64, n, u->ws, rows, use_lds, u->slabs);
    }
    hipLaunchKernelGGL(sum_slabs64_kernel, dim3(cdiv(nk, 16)), dim3(256), 0, v.stream, u->slabs, Gs, nk, u->sums);
    HCHK(hipGetLastError());
    if (trpo_dev_allreduce64(d, u->sums, (size_t)nk)) return -4;
    if (host_out) hipLaunchKernelGGL(copy64_kernel, dim3(1), dim3(64), 0, v.stream, (const double *)u->sums, host_out, nk);
    return 0;
}

extern "C" int trpo_dev_surrogate(trpo_dev *d, const double *fullstep, int k0, int nk, double *surr_host) {
    if (!d || !fullstep || !surr_host || k0 < 0 || nk < 1 || nk > 64 || k0 + nk > 1074) return -1;
    trpo_dev_view v;
    trpo_dev_get_view(d, &v);
    UpdState *u = state(d);
    if (!u->have_roll || u->roll_n != v.n) return -3;
    HCHK(hipSetDevice(v.device));
    const int P = v.net.P;
    if (!u->fs) HCHK(trpo_malloc((void **)&u->fs, sizeof(double) * P));
    // fullstep in through the mapped host buffer, the sums out through it
    if (ensure_host(u, (size_t)P + 64)) return -2;
    memcpy(u->hst, fullstep, sizeof(double) * P);
    hipLaunchKernelGGL(copy64_kernel, dim3(cdiv(P, 256)), dim3(256), 0, v.stream, (const double *)u->hst_dev, u->fs, P);
    int rc = enqueue_surrogate(d, u->fs, k0, nk);
    if (rc) return rc;
    hipLaunchKernelGGL(copy64_kernel, dim3(1), dim3(64), 0, v.stream, (const double *)u->sums, u->hst_dev + P, nk);
    HCHK(hipGetLastError());
    DSYNC(d);
    memcpy(surr_host, u->hst + P, sizeof(double) * nk);
    return 0;
}

// ===========================================================================
// Value-baseline objective for L-BFGS (reference src/TRPO_Baseline.c:29-240):
// per sample forward of the baseline MLP on [Obs, step / EpLen], output seed
// 0.02 (Predict - Target), backprop, gradient sums; fp64 like the policy-gradient
// generic kernel (N is small, ~3000, and L-BFGS wants consistent f and g).
// ===========================================================================
// THL: theta staged in LDS behind Y (round 5): read from global its wave-uniform loads are scalar loads,
// which return out of order, so every use waited for lgkmcnt(0) -- and with it for every LDS read in
// flight: the per-sample chains ran one memory round trip per multiply-add
template <bool LDSY, bool THL>
__global__ void __launch_bounds__(UT)
baseline_kernel(Net net, const double *__restrict__ thg, const double *__restrict__ obs,
                const double *__restrict__ target, int n, double *ws, int rows, int use_lds,
                double *__restrict__ slabs, double *__restrict__ pred) {
    extern __shared__ double lds64[];
    const int tid = threadIdx.x;
    // LDSY (compile time): with a run-time select hipcc cannot tell LDS from global and makes every
    // Y access a flat load / store (one lgkmcnt for LDS and the scalar theta loads alike: round 5)
    double *Y = LDSY ? lds64 : ws + (long)blockIdx.x * rows * RS;
    (void)use_lds;
    const double *th = thg;
    if constexpr (LDSY && THL) {
        double *tl = lds64 + rows * RS;
        for (int q = tid; q < net.P - net.A; q += UT) tl[q] = thg[q];
        __syncthreads();
        th = tl;
    }
    int roff[MAXL + 1];
    row_offsets(net, roff);
    const int tot = roff[net.nl], P = net.P, last = net.nl - 1;
    const int G0 = tot, GL = 2 * tot;          // gradient rows mirror Y's; then (y - t)^2 and a zero row
    int goff[MAXL];
    for (int i = 0; i + 1 < net.nl; ++i) goff[i] = G0 + roff[i + 1];
    double *slab = slabs + (long)blockIdx.x * (P + 1);
    const ThetaPlain T{th};
    for (int q = tid; q <= P; q += UT) slab[q] = 0.0;
    const int npass = (n + UT - 1) / UT;
    for (int pass = blockIdx.x; pass < npass; pass += gridDim.x) {
        const int s = pass * UT + tid;
        const bool live = s < n;
        forward64(net, T, obs, s, live, Y, roff, tid);
        const double y = Y[roff[last] * RS + tid];
        const double d = live ? y - target[s] : 0.0;
        if (live) pred[s] = y;                                         // :135
        Y[(G0 + roff[last]) * RS + tid] = 0.02 * d;                    // :140
        Y[GL * RS + tid] = d * d;
        Y[(GL + 1) * RS + tid] = 0.0;
        for (int i = last; i >= 1; --i) {                              // :143-188
            const int cur = net.L[i], a = net.act[i];
            for (int j = 0; j < cur; ++j) {
                const int e = (roff[i] + j) * RS + tid;
                Y[G0 * RS + e] = act_d64(a, Y[e], Y[G0 * RS + e]);
            }
            if (i >= 2) {
                const int prev = net.L[i - 1], wo = net.woff[i - 1];
                // FWD_JB outputs per sweep (independent chains, one read of each g_k for all of them;
                // each chain keeps its k-ascending order, so the sums are unchanged: round 5)
                int j = 0;
                for (; j + FWD_JB <= prev; j += FWD_JB) {
                    double t[FWD_JB];
#pragma unroll
                    for (int jj = 0; jj < FWD_JB; ++jj) t[jj] = 0.0;
#pragma unroll 16
                    for (int k = 0; k < cur; ++k) {
                        const double gk = Y[(G0 + roff[i] + k) * RS + tid];
#pragma unroll
                        for (int jj = 0; jj < FWD_JB; ++jj) t[jj] += gk * th[wo + (j + jj) * cur + k];
                    }
#pragma unroll
                    for (int jj = 0; jj < FWD_JB; ++jj) Y[(G0 + roff[i - 1] + j + jj) * RS + tid] = t[jj];
                }
                for (; j < prev; ++j) {
                    double t = 0.0;
#pragma unroll 4
                    for (int k = 0; k < cur; ++k) t += Y[(G0 + roff[i] + k) * RS + tid] * th[wo + j * cur + k];
                    Y[(G0 + roff[i - 1] + j) * RS + tid] = t;
                }
            }
        }
        __syncthreads();
        contract_pass(net, Y, roff, goff, GL, slab, tid);
        __syncthreads();
    }
}

// The same objective for the [L0, L1, L2, 1] baselines with L0, L1, L2 <= 16 (the trainer's [16, 16, 16, 1]),
// spread over lanes instead of down one lane's chain (round 5): baseline_kernel keeps a sample per lane,
// so one wave's ~1 100 dependent fp64 multiply-adds set the kernel time (60-65 us at any N; 46 us after
// its LDS fixes).  Here a 16-lane group works on one sample at a time, lane j owning neuron j of every
// layer: each dot product is a 16-step chain over values broadcast within the group (ds_bpermute),
// kept in the reference's order (bias first, inputs ascending; the backward sums from 0, ascending), so
// every per-sample value -- prediction, residual, activation gradients -- has the bits of
// baseline_kernel's.  Lane j accumulates its gradient entries (column j of W0 and W1, b0_j, b1_j, W2_j,
// and b2 and sum (y - t)^2) over the group's samples in sample order; the block's 16 groups are combined
// in group order through LDS into the block's slab (natural order, the layout baseline_kernel writes).
// Only the order of the sums over samples differs from baseline_kernel.
//
// Round 6: two launches per evaluate instead of three and no hipStreamSynchronize -- a small launch
// costs the host ~2.5 us to enqueue and the stream sync ~4.7 us more than spinning on pinned memory
// (tools/micro/host_wait, profiles/r06_host_wait.log):
//   - theta arrives BY VALUE in the kernel arguments (BlTheta, 4.5 KB: [16,16,16,1]'s 561 weights and
//     biases are the most this kernel takes; tools/micro/kernarg_big: +0.16 us of enqueue), no copy kernel;
//   - the slab sum (sum_slabs64_host_kernel) stores the sums into the pinned host buffer, each of its
//     blocks then its own flag word (the call's sequence number), and the host spins on the flags.
//     Summing the slabs in the same launch instead (the last block of each 16 sums their slabs, the
//     last group the partials, then one flag) was measured slower: 35 -> 58 us per evaluate with
//     agent-scope fences, 35 -> 43 us with fence-free `sc1` hand-offs -- each in-launch hand-off is a
//     drained store plus an atomic round trip, ~2 us apiece on this chip (profiles/r06_baseline_eval_ab.log).
constexpr int BLK_NE = 37;                 // per-lane accumulators: 16 W0, b0, 16 W1, b1, W2, b2, sum d^2
constexpr int BL_PA_MAX = 16 * 16 * 2 + 16 * 3 + 1;    // [16,16,16,1]: 561 weights and biases
struct BlTheta {
    double v[BL_PA_MAX];
};
__global__ void __launch_bounds__(256)
baseline_lane_kernel(Net net, BlTheta th, const double *__restrict__ obs, const double *__restrict__ target, int n,
                     double *__restrict__ slabs, double *__restrict__ pred) {
    __shared__ double tl[BL_PA_MAX + 1];                // theta (<= 16x16 + 16 + 16x16 + 16 + 16 + 1)
    __shared__ double acc[16][BLK_NE][16];              // [group][entry][lane]
    const int tid = threadIdx.x, lane = tid & 63, j = lane & 15, base = lane & ~15;
    const int gi = tid >> 4;                            // group in the block, 0..15
    const int L0 = net.L[0], L1 = net.L[1], L2 = net.L[2];
    const int a1 = net.act[1], a2 = net.act[2], a3 = net.act[3];
    const int W0 = net.woff[0], B0 = net.boff[0], W1 = net.woff[1], B1 = net.boff[1];
    const int W2 = net.woff[2], B2 = net.boff[2], PA = net.P - net.A;
    for (int q = tid; q < PA; q += 256) tl[q] = th.v[q];
    __syncthreads();
    double dw0[16], dw1[16], db0 = 0.0, db1 = 0.0, dw2 = 0.0, db2 = 0.0, fs = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) dw0[k] = dw1[k] = 0.0;
    const int ngroups = gridDim.x * 16;
    for (int s = blockIdx.x * 16 + gi; s < n; s += ngroups) {     // group-uniform trip count
        // forward (forward64's order: bias first, inputs ascending)
        const double xj = j < L0 ? obs[(long)s * L0 + j] : 0.0;
        double xk[16], y1k[16], y2k[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) xk[k] = __shfl(xj, base + k, 64);
        double z = j < L1 ? tl[B0 + j] : 0.0;
        for (int k = 0; k < L0; ++k) z += xk[k] * (j < L1 ? tl[W0 + k * L1 + j] : 0.0);
        const double y1 = j < L1 ? act_y64(a1, z) : 0.0;
#pragma unroll
        for (int k = 0; k < 16; ++k) y1k[k] = __shfl(y1, base + k, 64);
        z = j < L2 ? tl[B1 + j] : 0.0;
        for (int k = 0; k < L1; ++k) z += y1k[k] * (j < L2 ? tl[W1 + k * L2 + j] : 0.0);
        const double y2 = j < L2 ? act_y64(a2, z) : 0.0;
#pragma unroll
        for (int k = 0; k < 16; ++k) y2k[k] = __shfl(y2, base + k, 64);
        double z3 = tl[B2];
        for (int k = 0; k < L2; ++k) z3 += y2k[k] * tl[W2 + k];
        const double y3 = act_y64(a3, z3);
        const double d = y3 - target[s];
        if (pred && j == 0) __hip_atomic_store(pred + s, y3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);   // pinned
        // backward (baseline_kernel's order)
        const double g3 = act_d64(a3, y3, 0.02 * d);
        const double g2 = j < L2 ? act_d64(a2, y2, 0.0 + g3 * tl[W2 + j]) : 0.0;
        double g2k[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) g2k[k] = __shfl(g2, base + k, 64);
        double t = 0.0;
        for (int k = 0; k < L2; ++k) t += g2k[k] * (j < L1 ? tl[W1 + j * L2 + k] : 0.0);
        const double g1 = j < L1 ? act_d64(a1, y1, t) : 0.0;
        // this sample's gradient terms, lane j: column j of W0 and W1, b0_j, b1_j, W2_j; b2, d^2
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            dw0[k] += xk[k] * g1;
            dw1[k] += y1k[k] * g2;
        }
        db0 += g1;
        db1 += g2;
        dw2 += y2 * g3;
        db2 += g3;
        fs += d * d;
    }
    // the block's 16 groups in group order -> slab (natural order; then sum d^2, then a zero)
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        acc[gi][k][j] = dw0[k];
        acc[gi][17 + k][j] = dw1[k];
    }
    acc[gi][16][j] = db0;
    acc[gi][33][j] = db1;
    acc[gi][34][j] = dw2;
    acc[gi][35][j] = db2;
    acc[gi][36][j] = fs;
    __syncthreads();
    double *slab = slabs + (long)blockIdx.x * (net.P + 1);
    for (int q = tid; q <= net.P; q += 256) {
        int e = 36, l = 0;                             // q == PA: sum d^2 (lane 0); q == P: zero
        if (q < B0) { e = q / L1; l = q % L1; }
        else if (q < W1) { e = 16; l = q - B0; }
        else if (q < B1) { e = 17 + (q - W1) / L2; l = (q - W1) % L2; }
        else if (q < W2) { e = 33; l = q - B1; }
        else if (q < B2) { e = 34; l = q - W2; }
        else if (q < PA) { e = 35; l = 0; }
        double v = 0.0;
        if (q <= PA)
            for (int g = 0; g < 16; ++g) v += acc[g][e][l];
        slab[q] = v;
    }
}
// the slab sum of the evaluate (sum_slabs64_kernel's order) into pinned host memory; each block stores
// the call's sequence number into its own flag word behind its drained system-scope stores
__global__ void sum_slabs64_host_kernel(const double *__restrict__ slabs, int G, int len, double *__restrict__ out,
                                        unsigned *__restrict__ flags, unsigned seq) {
    __shared__ double part[16][17];
    const int tq = threadIdx.x & 15, tj = threadIdx.x >> 4;
    const int q = blockIdx.x * 16 + tq;
    double s = 0.0;
    if (q < len) {
#pragma unroll 8
        for (int b = tj; b < G; b += 16) s += slabs[(long)b * len + q];
    }
    part[tj][tq] = s;
    __syncthreads();
    if (tj == 0 && q < len) {
        double t = 0.0;
        for (int j = 0; j < 16; ++j) t += part[j][tq];
        __hip_atomic_store(out + q, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flags + blockIdx.x, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}


struct trpo_bdev {
    int device = 0;
    hipStream_t stream = nullptr;
    Net net;
    double *theta = nullptr, *obs = nullptr, *target = nullptr, *pred = nullptr;
    size_t n = 0, cap = 0;
    double *ws = nullptr;
    size_t ws_cap = 0;
    double *slabs = nullptr;
    size_t slab_cap = 0;
    double *sum = nullptr;
    int G = 1, rows = 0, use_lds = 0, lds = 0, theta_lds = 0;
    int lane_ok = 0, Gl = 1;                       // baseline_lane_kernel applies / its grid (round 5)
    double *hst = nullptr, *hst_dev = nullptr;   // pinned mapped host buffer: theta in, sums (+ predictions) out
    size_t hst_cap = 0;
    unsigned seq = 0;                            // the lane path's host hand-off: the last call's sequence number
    int started = 0, want_pred = 0;              // an eval_start without its eval_finish yet; with predictions
    size_t flag_at = 0;                          // where the flag words were zeroed last (they move with n)
};

static int act_code64(char a) {
    switch (a) {
    case 'l': return ACT_L;
    case 't': return ACT_T;
    case 'o': return ACT_O;
    case 's': return ACT_S;
    default: return -1;
    }
}

extern "C" void trpo_bdev_destroy(trpo_bdev *b) {
    if (!b) return;
    if (b->stream) hipStreamSynchronize(b->stream);
    void *ptrs[] = {b->theta, b->obs, b->target, b->pred, b->ws, b->slabs, b->sum};
    for (void *p : ptrs)
        if (p) hipFree(p);
    if (b->hst) hipHostFree(b->hst);
    if (b->stream) hipStreamDestroy(b->stream);
    delete b;
}

extern "C" trpo_bdev *trpo_bdev_create(int device, size_t nl, const size_t *ls, const char *ac, char *err,
                                       size_t errlen) {
    if (nl < 2 || nl > MAXL || !ls || !ac) {
        if (err) snprintf(err, errlen, "invalid baseline network (NumLayers=%zu)", nl);
        return nullptr;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        if (err) snprintf(err, errlen, "no HIP device available");
        return nullptr;
    }
    if (device < 0) {
        const char *e = getenv("TRPO_DEVICE");
        device = e ? atoi(e) : 0;
    }
    trpo_bdev *b = new trpo_bdev();
    b->device = device;
    Net &n = b->net;
    memset(&n, 0, sizeof n);
    n.nl = (int)nl;
    int pos = 0;
    for (size_t i = 0; i < nl; ++i) {
        n.L[i] = (int)ls[i];
        if (i > 0) n.act[i] = act_code64(ac[i]);
        if (ls[i] == 0 || (i > 0 && n.act[i] < 0)) {
            if (err) snprintf(err, errlen, "unsupported baseline layer %zu", i);
            delete b;
            return nullptr;
        }
    }
    for (size_t i = 0; i + 1 < nl; ++i) {
        n.woff[i] = pos;
        pos += n.L[i] * n.L[i + 1];
        n.boff[i] = pos;
        pos += n.L[i + 1];
    }
    n.A = n.L[nl - 1];
    n.P = pos + n.A;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking) != hipSuccess ||
        trpo_malloc((void **)&b->theta, sizeof(double) * n.P) != hipSuccess ||
        trpo_malloc((void **)&b->sum, sizeof(double) * (n.P + 1)) != hipSuccess) {
        if (err) snprintf(err, errlen, "baseline device allocation failed");
        trpo_bdev_destroy(b);
        return nullptr;
    }
    hipMemsetAsync(b->theta, 0, sizeof(double) * n.P, b->stream);
    b->rows = rows_for(n, false) * 2 + 2;
    const size_t bytes = sizeof(double) * (size_t)b->rows * RS, tbytes = sizeof(double) * (size_t)(n.P - n.A);
    b->use_lds = bytes <= (size_t)LDS_CAP;
    b->theta_lds = b->use_lds && bytes + tbytes <= (size_t)LDS_CAP;
    b->lds = b->use_lds ? (int)(bytes + (b->theta_lds ? tbytes : 0)) : 0;
    if (b->use_lds &&
        (hipFuncSetAttribute((const void *)baseline_kernel<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             LDS_CAP) != hipSuccess ||
         hipFuncSetAttribute((const void *)baseline_kernel<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             LDS_CAP) != hipSuccess)) {
        if (err) snprintf(err, errlen, "baseline LDS attribute failed");
        trpo_bdev_destroy(b);
        return nullptr;
    }
    return b;
}

// obs: [n][L0] including any extra input column(s) the caller appends (the time feature)
extern "C" int trpo_bdev_set_data(trpo_bdev *b, const double *obs, const double *target, size_t n) {
    if (!b || (n && (!obs || !target))) return -1;
    HCHK(hipSetDevice(b->device));
    const int L0 = b->net.L[0];
    if (n > b->cap) {
        if (b->obs) hipFree(b->obs);
        if (b->target) hipFree(b->target);
        if (b->pred) hipFree(b->pred);
        b->obs = b->target = b->pred = nullptr;
        b->cap = 0;
        HCHK(trpo_malloc((void **)&b->obs, sizeof(double) * n * L0));
        HCHK(trpo_malloc((void **)&b->target, sizeof(double) * n));
        HCHK(trpo_malloc((void **)&b->pred, sizeof(double) * n));
        b->cap = n;
    }
    b->n = n;
    b->G = n ? (cdiv((long)n, UT) < 1024 ? cdiv((long)n, UT) : 1024) : 1;
    // the lane-parallel kernel: [L0, L1, L2, 1] with widths <= 16; ~2 samples per 16-lane group
    const Net &nt = b->net;
    const char *el = getenv("TRPO_BASELINE_LANE");
    b->lane_ok = !(el && atoi(el) == 0) && nt.nl == 4 && nt.L[3] == 1 && nt.L[0] <= 16 && nt.L[1] <= 16 &&
                 nt.L[2] <= 16;
    // one sample per 16-lane group up to 256 blocks (round 6; 2 per group before: 31.3 -> 25.7 us per
    // evaluate at N = 3 000, profiles/r06_baseline_eval_ab.log)
    b->Gl = n ? (cdiv((long)n, 16) < 256 ? (int)cdiv((long)n, 16) : 256) : 1;
    const int gs = b->lane_ok && b->Gl > b->G ? b->Gl : b->G;
    if (ensure(&b->slabs, &b->slab_cap, (size_t)gs * (b->net.P + 1), b->stream)) return -2;
    if (!b->use_lds && ensure(&b->ws, &b->ws_cap, (size_t)b->rows * RS * b->G, b->stream)) return -2;
    if (n) {
        HCHK(hipMemcpyAsync(b->obs, obs, sizeof(double) * n * L0, hipMemcpyHostToDevice, b->stream));
        HCHK(hipMemcpyAsync(b->target, target, sizeof(double) * n, hipMemcpyHostToDevice, b->stream));
    }
    HCHK(hipStreamSynchronize(b->stream));
    return 0;
}


// theta: natural [W, B per layer] (P - A values); gsum[P + 1]: gradient sums (P - A entries),
// then sum (y - t)^2 at P - A; pred (n, may be NULL) receives the predictions
// trpo_bdev_eval in two halves, so that a caller can do host work while the device evaluates
// (evaluate()'s comparison of the caller's arrays, trpo_host.c): _start enqueues, _finish waits and
// copies out; every _start must be followed by one _finish.  want_pred: the predictions are produced.
extern "C" int trpo_bdev_eval_start(trpo_bdev *b, const double *theta, int want_pred) {
    if (!b || !theta || !b->n || b->started) return -1;
    HCHK(hipSetDevice(b->device));
    const Net &net = b->net;
    const int P = net.P;
    // x in and (f, g[, predictions]) out through pinned device-mapped host memory, moved by small
    // kernels: no pageable copies on the L-BFGS callback's critical path
    // [f, g | predictions | theta in | the slab sum's per-block flags]
    const int nfl = cdiv(P + 1, 16);
    const size_t need = (size_t)P + 1 + b->n + (size_t)(P - net.A) + cdiv(nfl, 2);
    if (need > b->hst_cap) {
        if (b->hst) hipHostFree(b->hst);
        b->hst = b->hst_dev = nullptr;
        b->hst_cap = 0;
        HCHK(hipHostMalloc((void **)&b->hst, sizeof(double) * need, TRPO_HOST_COHERENT));
        HCHK(hipHostGetDevicePointer((void **)&b->hst_dev, b->hst, 0));
        b->hst_cap = need;
        memset(b->hst, 0, sizeof(double) * need);
    }
    if (b->lane_ok && P - net.A <= BL_PA_MAX) {
        // theta by value, the sums (and the predictions) straight into the pinned buffer, a spin on the
        // slab sum's flags (baseline_lane_kernel)
        BlTheta th;
        memcpy(th.v, theta, sizeof(double) * (P - net.A));
        if (++b->seq == 0) b->seq = 1;
        const size_t foff = (size_t)P + 1 + b->n + (size_t)(P - net.A);
        if (foff != b->flag_at) {                  // a new layout: no stale word may read as this seq
            memset(b->hst + foff, 0, sizeof(double) * cdiv(nfl, 2));
            b->flag_at = foff;
        }
        hipLaunchKernelGGL(baseline_lane_kernel, dim3(b->Gl), dim3(256), 0, b->stream, net, th, (const double *)b->obs,
                           (const double *)b->target, (int)b->n, b->slabs, want_pred ? b->hst_dev + P + 1 : nullptr);
        hipLaunchKernelGGL(sum_slabs64_host_kernel, dim3(nfl), dim3(256), 0, b->stream, (const double *)b->slabs, b->Gl,
                           P + 1, b->hst_dev, (unsigned *)(b->hst_dev + foff), b->seq);
        HCHK(hipGetLastError());
        b->started = 1;
        b->want_pred = want_pred;
        return 0;
    }
    double *hin = b->hst + P + 1 + b->n;                   // theta staging after the outputs
    memcpy(hin, theta, sizeof(double) * (P - net.A));
    hipLaunchKernelGGL(copy64_kernel, dim3(cdiv(P - net.A, 256)), dim3(256), 0, b->stream,
                       (const double *)(b->hst_dev + P + 1 + b->n), b->theta, P - net.A);
    const int gsl = b->G;
    {
        void (*bk)(Net, const double *, const double *, const double *, int, double *, int, int, double *, double *) =
            b->theta_lds ? baseline_kernel<true, true>
                         : (b->use_lds ? baseline_kernel<true, false> : baseline_kernel<false, false>);
        hipLaunchKernelGGL(bk, dim3(b->G), dim3(UT), b->lds, b->stream, net, (const double *)b->theta,
                           (const double *)b->obs, (const double *)b->target, (int)b->n, b->ws, b->rows, b->use_lds,
                           b->slabs, b->pred);
    }
    // the sums go straight into the mapped host buffer (round 5: one copy launch fewer per callback)
    hipLaunchKernelGGL(sum_slabs64_kernel, dim3(cdiv(P + 1, 16)), dim3(256), 0, b->stream, b->slabs, gsl, P + 1,
                       b->hst_dev);
    if (want_pred)
        hipLaunchKernelGGL(copy64_kernel, dim3(cdiv((long)b->n, 256)), dim3(256), 0, b->stream, (const double *)b->pred,
                           b->hst_dev + P + 1, (int)b->n);
    HCHK(hipGetLastError());
    b->started = 1;
    b->want_pred = want_pred;
    return 0;
}

extern "C" int trpo_bdev_eval_finish(trpo_bdev *b, double *gsum, double *pred) {
    if (!b || !gsum || !b->started || (pred && !b->want_pred)) return -1;
    b->started = 0;
    HCHK(hipSetDevice(b->device));
    const Net &net = b->net;
    const int P = net.P;
    if (b->lane_ok && P - net.A <= BL_PA_MAX) {
        const size_t foff = (size_t)P + 1 + b->n + (size_t)(P - net.A);
        if (const int rc = trpo_wait_host_flags(b->stream, (const unsigned *)(b->hst + foff), cdiv(P + 1, 16), b->seq, 100))
            return rc;
    } else {
        HCHK(hipStreamSynchronize(b->stream));
    }
    memcpy(gsum, b->hst, sizeof(double) * (P + 1));
    if (pred) memcpy(pred, b->hst + P + 1, sizeof(double) * b->n);
    return 0;
}

extern "C" int trpo_bdev_eval(trpo_bdev *b, const double *theta, double *gsum, double *pred) {
    if (!gsum) return -1;
    const int rc = trpo_bdev_eval_start(b, theta, pred != nullptr);
    return rc ? rc : trpo_bdev_eval_finish(b, gsum, pred);
}
