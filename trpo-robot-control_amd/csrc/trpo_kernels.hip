// trpo_kernels.hip -- gfx950 (MI355X / CDNA4) kernels for the TRPO Fisher-vector
// product and the conjugate-gradient solve, plus the device layer behind
// trpo_dev.h.
//
// Math (reference src/TRPO_FVP.c:548-949, FVPFast):
//   per sample n:  forward  y_{i+1} = act(W_i^T y_i + b_i)
//                  R-fwd    Rx_{i+1} = W_i^T Ry_i + VW_i^T y_i + vb_i,  Ry = act'(.) Rx
//                  R-bwd    G_L = act_L'(Ry_L / sigma^2),  G_i = act_i'(W_i G_{i+1})
//   Fv = (1/N) sum_n [ y_i (x) G_{i+1} ; G_{i+1} ]  +  [2 v_logstd]  +  damping * v
//
// MI355X mapping:
//   * 16 samples = one tile; a wave streams tiles.  All layer products run on
//     v_mfma_f32_16x16x4_f32 in the TRANSPOSED orientation: neurons on MFMA
//     rows, samples on columns, so each layer's accumulator registers ARE the
//     next layer's B operand (k permuted: lane group g, step s <-> neuron 4g+s)
//     -- no data movement between layers, forward or backward.
//   * the cross-sample contraction sum_n y (x) G is an MFMA with K = samples;
//     its operands are transposed through a 20-float-stride per-wave LDS
//     scratch (4 ds_write_b32 + 1 ds_read_b128 per 16x16 tile).
//   * weights (and VW = the direction being multiplied) are staged in LDS in
//     MFMA-fragment order, read with ds_read_b128 (lane-contiguous, conflict
//     free); the fp64 direction is gathered+converted into LDS per block.
//   * per-block fp32 partials are combined across the block's waves by a
//     fixed pairwise tree (deterministic), then reduced across blocks in fp64
//     by a second kernel in a fixed order.  CG scalars and vectors are fp64.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>
#include <math.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "trpo_common.h"
#include "trpo_dev.h"

typedef float f4 __attribute__((ext_vector_type(4)));

#define MFMA(a, b, c) __builtin_amdgcn_mfma_f32_16x16x4f32((a), (b), (c), 0, 0, 0)
// v_mfma_f32_4x4x1_16b_f32: 16 blocks of 4x4 with K = 1; lane l is block l / 4, supplies A_b[l % 4] and
// B_b[l % 4], and register i of lane 4b + j accumulates A_b[i] B_b[j] (probed: tools/micro/mfma4x4.hip)
#define MFMA4(a, b, c) __builtin_amdgcn_mfma_f32_4x4x1f32((a), (b), (c), 0, 0, 0)

// Fragment-order pack layout for the 3-weight-layer fast path (offsets in floats).
struct Pack {
    int T[4];                  // tiles of 16 per layer: T0 (input) .. T3 (output)
    int fa[3], fb[3], bi[3], iv, tlen;
    int vfa[3], vb[3], vlen;
};

struct Ctl {                   // device-side control block of one context
    double damping;
    double n_total;
    double resth;
    double rdotr;
    int maxiter;
    int iter;
    int done;
    int zero;                  // always 0: "never skip" flag for standalone FVPs
    double orth;               // max over the solve's steps of the fraction of |r'|^2 the residual
                               // reorthogonalisation removed (sum c^2 / |r'|^2)
    double alpha[64];          // the step lengths alpha_k of the first 64 steps (CG_AMAX): with the
                               // rdotr history they give the Lanczos matrix of the solve, whose Ritz
                               // residuals are the fp32 stall guard's test (trpo_host.c)
};
constexpr int CG_AMAX = 64;
static_assert(offsetof(Ctl, alpha) == offsetof(Ctl, orth) + sizeof(double) && TRPO_CG_STATS == 1 + CG_AMAX,
              "Ctl: orth, alpha[] contiguous (one copy exports the statistics)");

// block 0, one lane: ctl->orth = max(ctl->orth, cs / |r'|^2) with |r'|^2 = |r''|^2 + cs
__device__ __forceinline__ void note_orth(double *orth, double cs, double nr) {
    const double tot = nr + cs;
    const double f = tot > 0.0 ? cs / tot : 0.0;
    *orth = f > *orth ? f : *orth;
}

struct CgSt {                  // ping-ponged CG scalars (state k = before FVP k)
    double rdotr;
    double xx;                 // |x|^2 (printed as the "Soln Norm")
    int iter;
    int pad;
};

// Arguments of one fused FVP / CG-iteration launch.
struct IterArgs {
    const float4 *obs4;
    int n, ntiles, P, nw;
    int Ps;                       // even row stride of the replica sets and the basis (P rounded up)
    const float *tpack;
    const float *vpack;           // plain FVP: the packed direction
    const double *v_nat;          // plain FVP: gather the direction from this natural-order vector instead
    float *slabs;                 // slab epilogue (acc_out == nullptr)
    double *acc_out;              // atomic epilogue: R_out fp64 replicas of the P-vector
    int R_out;
    double *acc_zero;             // buffer zeroed by block 0 (next-but-one accumulation target)
    int zero_len;
    const int *imap;              // slab/accumulator position -> natural parameter
    const int *skip;
    // fused CG update prologue (update != 0): z = sum(acc_in)/N + lambda p ; one CG step
    int update;
    const double *acc_in;
    int R_in;
    const double *p_in, *r_in;
    double *p_out, *r_out, *x;
    const CgSt *st_in;
    CgSt *st_out;
    Ctl *ctl;
    double *hist;
    const int *vmap;
    // policy-gradient mode (MODE == 1, src/TRPO_Update.c:254-378): per padded sample the
    // fp32 (Action - Mean) rows [16 T3] and Adv, and 1/sigma^2 with sigma = exp(LogStd)
    const float4 *pg_d4;
    const float *pg_adv;
    const float4 *pg_iv4;
    // forward-activation cache [tile][T1 + T2 + T3][lane] f4 (the per-tile y1, y2, y3 in D-layout):
    // MODE 0 writes it when non-null, MODE 2 reads it instead of recomputing the forward pass
    float4 *yc;
    // CG start fused into the first FVP of a solve (init != 0, src/TRPO_CG.c:24-40): the direction
    // is p0 = b (b_init, natural order); the last block writes x = 0, r = p = b, rdotr = b.b, the
    // state and the control block (maxiter, resth, done) -- replaces a separate init launch
    int init, init_maxiter;
    double init_resth;
    const double *b_init;
    const int *pslot;             // natural parameter -> v-pack slot (pslot_at), -1 for LogStd
    const int *islot;             // natural parameter -> slab / accumulator position (islot_at), [nw]
    // residual reorthogonalisation (update / init): the basis q_0 .. q_{QCAP-1} (fp64 [QCAP][P]), the
    // number of stored vectors this step uses (nq = min(iteration before the step, QCAP)), a zero line,
    // and whether reorthogonalisation is on (TRPO_CG_REORTH, default 1)
    void *q;                      // QT [QCAP][P]: float (fp32 kernels) or double (fp64 mode)
    const void *qz;
    int nq, reorth;
    int gmaj;                     // cooperative kernel: group-major tile order (TRPO_COOP_GMAJ)
};

// fixed-order block-wide fp64 sum (every thread gets the result)
__device__ double block_sum(double v, double *sh) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nwv = blockDim.x >> 6;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    __syncthreads();
    if (lane == 0) sh[w] = v;
    __syncthreads();
    double t = 0.0;
    for (int k = 0; k < nwv; ++k) t += sh[k];
    return t;
}

// fp64 DPP row (16-lane) sum; every lane of the row gets it.  Fixed order => deterministic.
template <int CTRL>
__device__ __forceinline__ double dpp64(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double rowsum16_f64(double v) {
    v += dpp64<0xB1>(v);    // quad_perm xor 1
    v += dpp64<0x4E>(v);    // quad_perm xor 2
    v += dpp64<0x124>(v);   // row_ror 4
    v += dpp64<0x128>(v);   // row_ror 8
    return v;
}
__device__ __forceinline__ double readlane64(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// fp64 half exchanges across a wave (gfx950 v_permlane32_swap / v_permlane16_swap, one per dword):
// swap32: lanes 32-63 of a <-> lanes 0-31 of b;  swap16: odd 16-lane rows of a <-> even rows of b
__device__ __forceinline__ void swap32_f64(double &a, double &b) {
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)__double2loint(a), (unsigned)__double2loint(b), false,
                                                     false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)__double2hiint(a), (unsigned)__double2hiint(b), false,
                                                     false);
    a = __hiloint2double((int)hi[0], (int)lo[0]);
    b = __hiloint2double((int)hi[1], (int)lo[1]);
}
__device__ __forceinline__ void swap16_f64(double &a, double &b) {
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)__double2loint(a), (unsigned)__double2loint(b), false,
                                                     false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)__double2hiint(a), (unsigned)__double2hiint(b), false,
                                                     false);
    a = __hiloint2double((int)hi[0], (int)lo[0]);
    b = __hiloint2double((int)hi[1], (int)lo[1]);
}
// block-wide fp64 sums of K values (blocks of W waves, W <= 16) with ONE barrier; every thread gets
// the K totals (wave-uniform).  Per wave a transpose-reduce: the K values (padded to KP = 4, 8, 16
// or 32) are halved twice across the half-waves and the 16-lane rows by permlane swaps -- each step
// adds lane l and its partner in a fixed order and leaves half the values per lane -- then each of
// the KP/4 registers is summed over its rows with DPP; row r of register k then holds the wave's
// total of value k + (r & 1) KP/4 + (r >> 1) KP/2.  Those go to LDS ([wave][value]); after the
// barrier lane v sums value v over the waves in wave order and the totals are read out of lanes.
// Fixed order throughout, so every wave and block gets bit-identical totals.  ~2K + 8 VALU
// cross-lane steps per wave instead of 12K for K separate DPP+readlane reductions.
// sh must hold W * KP doubles and must not be reused by another call before the block passes
// another barrier.
template <int K, int W>
__device__ __forceinline__ void block_sums_dpp(double (&v)[K], double *sh) {
    static_assert(K >= 1 && K <= 32 && W >= 1 && W <= 16, "block_sums_dpp");
    constexpr int KP = K <= 4 ? 4 : K <= 8 ? 8 : K <= 16 ? 16 : 32;
    constexpr int H = KP / 2, Q = KP / 4;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, row = lane >> 4;
    double t[KP];
#pragma unroll
    for (int k = 0; k < KP; ++k) t[k] = k < K ? v[k] : 0.0;
#pragma unroll
    for (int k = 0; k < H; ++k) {               // lanes 0-31: value k, lanes 32-63: value k + H
        swap32_f64(t[k], t[k + H]);
        t[k] = t[k] + t[k + H];
    }
#pragma unroll
    for (int k = 0; k < Q; ++k) {               // rows 0..3: values k, k + Q, k + H, k + Q + H
        swap16_f64(t[k], t[k + Q]);
        t[k] = t[k] + t[k + Q];
    }
#pragma unroll
    for (int k = 0; k < Q; ++k) t[k] = rowsum16_f64(t[k]);
    if ((lane & 15) == 0) {
        const int off = w * KP + (row & 1) * Q + (row >> 1) * H;
#pragma unroll
        for (int k = 0; k < Q; ++k) sh[off + k] = t[k];
    }
    __syncthreads();
    const int vv = lane & (KP - 1);
    double s = sh[vv];
#pragma unroll
    for (int ww = 1; ww < W; ++ww) s += sh[ww * KP + vv];
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = readlane64(s, k);
}

// one value through block_sums_dpp's per-wave tree (lane l + lane l+32, then + the next row, then the
// DPP row sum): the result in lane 0 equals the wave total block_sums_dpp forms for any value, so
// the streaming basis dots below reproduce its bits
__device__ __forceinline__ double wave_tree_sum(double v) {
    double a = v, b = v;
    swap32_f64(a, b);
    a = a + b;
    b = a;
    swap16_f64(a, b);
    a = a + b;
    return rowsum16_f64(a);
}

// two fixed-order block-wide fp64 sums at once (sh: 2 x 16 doubles)
__device__ void block_sum2(double a, double b, double *sh, double &sa, double &sb) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nwv = blockDim.x >> 6;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        a += __shfl_xor(a, off, 64);
        b += __shfl_xor(b, off, 64);
    }
    __syncthreads();
    if (lane == 0) {
        sh[w] = a;
        sh[16 + w] = b;
    }
    __syncthreads();
    double ta = 0.0, tb = 0.0;
    for (int k = 0; k < nwv; ++k) {
        ta += sh[k];
        tb += sh[16 + k];
    }
    sa = ta;
    sb = tb;
}

// ---------------------------------------------------------------------------
// Residual reorthogonalisation of the CG step.  The fp32 FVP returns F p + delta(p) with
// |delta| ~ 1e-7 |F p| and delta a NON-linear function of p, so CG's residuals lose their mutual
// orthogonality and the 10-step iterate drifts from the fp64 reference's by up to ~1e-3
// (tools/cg_noise_variants.py).  Each step therefore removes from the new residual
// r' = r - alpha z its components along the normalised earlier residuals q_i = r_i / |r_i| (classical
// Gram-Schmidt, fp64): c_i = q_i . r' = -alpha q_i . z for the stored basis (r is orthogonal to it
// after the previous step) and c = |r| - alpha (r . z) / |r| along the current residual itself, so
// only the dots q_i . z join the step's block reduction.  In exact arithmetic every c is zero, so the
// iterates are the reference's (src/TRPO_CG.c:65-103); with the fp32 FVP the step lands within 1e-7 of
// the fp64 reference instead of 1e-3.  |r''|^2 = |r'|^2 - sum c^2.  The basis q_0 .. q_{QCAP-1} lives in
// HBM (natural order); longer solves are reorthogonalised against the first QCAP residuals.
// Basis element type QT: fp32 in the fp32-FVP paths, fp64 in the fp64 precision mode.  An fp32
// basis is enough where the FVP itself carries fp32 noise: the projection then removes the
// components along fl32(q_i), which leaves r'' orthogonal to the true q_i to ~3e-9 |r''| (against
// ~1e-7 without reorthogonalisation), and the numpy emulation (tools/cg_noise_variants.py) lands
// on the fp64-basis step to 3 digits on every CG / update golden; it halves the basis bytes every
// block of the CG-iteration kernel loads in its prologue.  In the fp64 mode the fp32 rounding of
// the basis (6e-8) would itself exceed the FVP noise, so that mode keeps fp64.
// ---------------------------------------------------------------------------
constexpr int QCAP = 16;
// fp64 atomic replica sets of the small-net FVP partial sums: at most RMAX, RMAX by
// default (6 measured 1.6 % faster than 8 and 4 at N = 50k / 6 250: fewer prologue loads against
// more adds per address)
constexpr int RMAX = 6;

// the thread's E elements (q = tid + e * nthreads) of basis vector i, or zeros for i >= nq / q >= P:
// the load is unconditional (a select on the address: qz is a small zero line every lane may read)
// Element layouts of the P-vectors in the CG steps: thread t holds elements t + e * nthreads, or with
// PAIR (two elements per thread, P <= 2 * nthreads) the adjacent pair 2t, 2t + 1, loaded by one
// 16-byte (8-byte for fp32) instruction -- narrow loads issue at about half the byte rate.
// Replica and basis rows have the even stride Ps, so every pair is aligned.
template <bool PAIR>
__device__ __forceinline__ int elem_of(int e, int nthreads) {
    return PAIR ? 2 * (int)threadIdx.x + e : (int)threadIdx.x + e * nthreads;
}
template <typename T> struct V2T;
template <> struct V2T<float> { typedef float2 type; };
template <> struct V2T<double> { typedef double2 type; };
template <> struct V2T<int> { typedef int2 type; };
// the pair (2t, 2t + 1) of row `row` (stride Ps) of base, clamped to a valid pair (values selected by
// the caller); one vector load
template <typename T>
__device__ __forceinline__ typename V2T<T>::type pair_at(const T *base, long row, int Ps) {
    const int t = min((int)threadIdx.x, (Ps >> 1) - 1);
    return reinterpret_cast<const typename V2T<T>::type *>(base + row * Ps)[t];
}

template <int E, typename QT, bool PAIR = false>
__device__ __forceinline__ void qload(double (&dst)[E], const QT *Q, const QT *qz, int P, int Ps, int i, int nq,
                                      int nthreads) {
    const int tid = threadIdx.x;
    if constexpr (PAIR) {
        static_assert(E == 2, "pair layout");
        const bool ok = i < nq;
        typedef typename V2T<QT>::type V2;
        const V2 *src = ok ? reinterpret_cast<const V2 *>(Q + (long)i * Ps) + min(tid, (Ps >> 1) - 1)
                           : reinterpret_cast<const V2 *>(qz) + (tid & 7);
        const V2 v = *src;
        dst[0] = (ok && 2 * tid < P) ? (double)v.x : 0.0;
        dst[1] = (ok && 2 * tid + 1 < P) ? (double)v.y : 0.0;
        return;
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int q = tid + e * nthreads;
        const bool ok = i < nq && q < P;
        const QT *src = ok ? Q + (long)i * Ps + q : qz + (tid & 7);
        const double v = (double)*src;
        dst[e] = ok ? v : 0.0;
    }
}

// stage 1 of the dots e_i = q_i . z, i < nq (runtime): per wave the total by block_sums_dpp's tree,
// written to shq[i * W + w]; a later barrier (the caller's block reduction) makes them visible.
// Loads of the next vector are issued before the current one is reduced.
template <int E, typename QT, bool PAIR = false>
__device__ void qdots_stage1(const QT *Q, const QT *qz, int P, int Ps, int nq, const double (&zv)[E], int nthreads,
                             double *shq) {
#pragma clang fp contract(off)
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    if constexpr (E > 4) {          // many elements per thread: one vector at a time (register budget)
        for (int i = 0; i < nq; ++i) {
            double qa[E];
            qload<E, QT, PAIR>(qa, Q, qz, P, Ps, i, nq, nthreads);
            double t = 0.0;
#pragma unroll
            for (int e = 0; e < E; ++e) t = __builtin_fma(qa[e], zv[e], t);
            t = wave_tree_sum(t);
            if (lane == 0) shq[i * nwv + w] = t;
        }
        return;
    }
    double qa[E], qb[E];
    qload<E, QT, PAIR>(qa, Q, qz, P, Ps, 0, nq, nthreads);
    for (int i = 0; i < nq; i += 2) {
        qload<E, QT, PAIR>(qb, Q, qz, P, Ps, i + 1, nq, nthreads);
        double t = 0.0;
#pragma unroll
        for (int e = 0; e < E; ++e) t = __builtin_fma(qa[e], zv[e], t);
        t = wave_tree_sum(t);
        if (lane == 0) shq[i * nwv + w] = t;
        qload<E, QT, PAIR>(qa, Q, qz, P, Ps, i + 2, nq, nthreads);
        if (i + 1 < nq) {
            t = 0.0;
#pragma unroll
            for (int e = 0; e < E; ++e) t = __builtin_fma(qb[e], zv[e], t);
            t = wave_tree_sum(t);
            if (lane == 0) shq[(i + 1) * nwv + w] = t;
        }
    }
}

// stage 2: e_i from the wave totals in wave order -- block_sums_dpp's order (after a barrier)
__device__ __forceinline__ double qdot_final(const double *shq, int i) {
    const int nwv = blockDim.x >> 6;
    double s = shq[i * nwv];
    for (int w = 1; w < nwv; ++w) s += shq[i * nwv + w];
    return s;
}

// stage 3: rv -= sum_i c_i q_i with c_i = -alpha e_i (i < nq); returns sum_i c_i^2
template <int E, typename QT, bool PAIR = false>
__device__ double qcorrect(const QT *Q, const QT *qz, int P, int Ps, int nq, int nthreads, const double *shq,
                           double alpha, double (&rv)[E]) {
#pragma clang fp contract(off)
    if constexpr (E > 4) {          // register budget, as qdots_stage1
        double cs = 0.0;
        for (int i = 0; i < nq; ++i) {
            double qa[E];
            qload<E, QT, PAIR>(qa, Q, qz, P, Ps, i, nq, nthreads);
            const double c = -alpha * qdot_final(shq, i);
            cs += c * c;
#pragma unroll
            for (int e = 0; e < E; ++e) rv[e] = __builtin_fma(-c, qa[e], rv[e]);
        }
        return cs;
    }
    double qa[E], qb[E], cs = 0.0;
    qload<E, QT, PAIR>(qa, Q, qz, P, Ps, 0, nq, nthreads);
    for (int i = 0; i < nq; i += 2) {
        qload<E, QT, PAIR>(qb, Q, qz, P, Ps, i + 1, nq, nthreads);
        double c = -alpha * qdot_final(shq, i);
        cs += c * c;
#pragma unroll
        for (int e = 0; e < E; ++e) rv[e] = __builtin_fma(-c, qa[e], rv[e]);
        qload<E, QT, PAIR>(qa, Q, qz, P, Ps, i + 2, nq, nthreads);
        if (i + 1 < nq) {
            c = -alpha * qdot_final(shq, i + 1);
            cs += c * c;
#pragma unroll
            for (int e = 0; e < E; ++e) rv[e] = __builtin_fma(-c, qb[e], rv[e]);
        }
    }
    return cs;
}

// block 0 stores the new basis vector q_it = r'' / |r''| (it < QCAP)
template <int E, typename QT, bool PAIR = false>
__device__ __forceinline__ void qstore(QT *Q, int P, int Ps, int it, double nr, const double (&rv)[E],
                                       int nthreads) {
    if (!Q || it >= QCAP) return;
    const double inv = nr > 0.0 ? 1.0 / sqrt(nr) : 0.0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int q = elem_of<PAIR>(e, nthreads);
        if (q < P) Q[(long)it * Ps + q] = (QT)(rv[e] * inv);
    }
}

// ---------------------------------------------------------------------------
// activation helpers (reference src/TRPO_FVP.c:810-834 and :866-882)
// ---------------------------------------------------------------------------
// fp32 tanh for the tile kernel: |x| < 0.625 odd polynomial x(1 + x^2 Q(x^2)) (Chebyshev-node
// least squares, degree 4), else 1 - 2 / (e^{2|x|} + 1) with the hardware exp2 / rcp.  Max
// relative error 1.5e-7 (tools/fit_tanh.py), 14 VALU ops against ~22 for the libm tanhf; the tile
// loop is VALU+MFMA issue bound, so this is time.  Same function in every FVP => the small
// deviation from tanhf is a fixed perturbation of F, not noise across CG iterations.
__device__ __forceinline__ float tanh_fast(float x) {
    const float ax = fabsf(x), u = x * x;
    float q = fmaf(u, -0.006104945205152035f, 0.021003639325499535f);
    q = fmaf(u, q, -0.05385249853134155f);
    q = fmaf(u, q, 0.13332782685756683f);
    q = fmaf(u, q, -0.333333283662796f);
    const float ts = fmaf(ax * u, q, ax);
    const float e = __builtin_amdgcn_exp2f(ax * 2.8853900817779268f);      // e^{2|x|}
    const float tb = fmaf(-2.0f, __builtin_amdgcn_rcpf(e + 1.0f), 1.0f);
    return copysignf(ax < 0.625f ? ts : tb, x);
}
// fp32 logistic 1 / (1 + e^{-x}) with the hardware exp2 / rcp
__device__ __forceinline__ float sigmoid_fast(float x) {
    return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.4426950408889634f));
}
__device__ __forceinline__ float act_y(int a, float x) {
    switch (a) {
    case ACT_T: return tanhf(x);
    case ACT_O: return 0.1f * x;
    case ACT_S: return 1.0f / (1.0f + expf(-x));
    default: return x;
    }
}
// R{y} from R{x} given y
__device__ __forceinline__ float act_r(int a, float y, float rx) {
    switch (a) {
    case ACT_T: return rx * (1.0f - y * y);
    case ACT_O: return 0.1f * rx;
    case ACT_S: return rx * y * (1.0f - y);
    default: return rx;
    }
}
// fp64 twins (the generic kernel's precision mode): tanh64 (trpo_common.h) and the libm exp
__device__ __forceinline__ double act_y(int a, double x) {
    switch (a) {
    case ACT_T: return tanh64(x);
    case ACT_O: return 0.1 * x;
    case ACT_S: return 1.0 / (1.0 + exp(-x));
    default: return x;
    }
}
__device__ __forceinline__ double act_r(int a, double y, double rx) {
    switch (a) {
    case ACT_T: return rx * (1.0 - y * y);
    case ACT_O: return 0.1 * rx;
    case ACT_S: return rx * y * (1.0 - y);
    default: return rx;
    }
}
// tanh' = 1 - y^2 as ONE explicit fma: left to the compiler, whether the product is fused
// depends on what else uses y*y, so the recomputing (MODE 0) and cached (MODE 2) kernels could
// round it differently -- they must agree bit for bit
__device__ __forceinline__ float dtanh(float y) { return __builtin_fmaf(-y, y, 1.0f); }
__device__ __forceinline__ f4 dtanh4(f4 y) {
    f4 d;
#pragma unroll
    for (int r = 0; r < 4; ++r) d[r] = dtanh(y[r]);
    return d;
}
__device__ __forceinline__ f4 act_fwd(int a, f4 x, f4 rx, f4 &ry) {
    f4 y;
    if (a == ACT_T) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            y[r] = tanh_fast(x[r]);
            ry[r] = rx[r] * dtanh(y[r]);
        }
    } else if (a == ACT_S) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            y[r] = sigmoid_fast(x[r]);
            ry[r] = rx[r] * y[r] * (1.0f - y[r]);
        }
    } else if (a == ACT_O) {
        y = 0.1f * x;
        ry = 0.1f * rx;
    } else {
        y = x;
        ry = rx;
    }
    return y;
}
__device__ __forceinline__ f4 act_bwd(int a, f4 y, f4 g) {
    if (a == ACT_T) return g * (1.0f - y * y);
    if (a == ACT_S) return g * y * (1.0f - y);
    if (a == ACT_O) return 0.1f * g;
    return g;
}
__host__ __device__ constexpr inline bool act_needs_y(int a) { return a == ACT_T || a == ACT_S; }
// R{y} of four rows from R{x} and the (cached) forward value y
__device__ __forceinline__ f4 act_r4(int a, f4 y, f4 rx) {
    if (a == ACT_T) return rx * dtanh4(y);
    if (a == ACT_S) return rx * y * (1.0f - y);
    if (a == ACT_O) return 0.1f * rx;
    return rx;
}

// ---------------------------------------------------------------------------
// pack-slot -> natural-parameter maps (built once per context)
// ---------------------------------------------------------------------------
// theta pack: FA_i[ot][kt][lane][s] = W_i[16kt+4g+s][16ot+c]
//             FB_i[it][kt][lane][s] = W_i[16it+c][16kt+4g+s]   (i = 1, 2)
//             BI_i[j] = b_i[j];  IV[j] = 1/sigma_j^2 (filled separately)
// v pack:     VFA_i like FA_i, VB_i like BI_i
// p64: fp64 packs (v_mfma_f64_16x16x4_f64 keeps row g + 4s where the f32 MFMA keeps 4g + s)
__device__ int map_frag(const Net &n, int i, int local, int nkt, bool fwd, bool p64 = false) {
    const int idx4 = local >> 2, s = local & 3, lane = idx4 & 63, tk = idx4 >> 6;
    const int kt = tk % nkt, ot = tk / nkt, g = lane >> 4, c = lane & 15;
    const int ks = p64 ? g + 4 * s : 4 * g + s;
    int in, out;
    if (fwd) { in = 16 * kt + ks; out = 16 * ot + c; }
    else     { in = 16 * ot + c;  out = 16 * kt + ks; }
    if (in >= n.L[i] || out >= n.L[i + 1]) return -1;
    return n.woff[i] + in * n.L[i + 1] + out;
}

// v-pack slot -> natural parameter (or -1).  Pure integer math on the shape, so the fused
// kernel evaluates it in registers instead of loading a map (T compile-time there).
__device__ __forceinline__ int vmap_at(const Net &n, const int (&T)[4], int e, bool p64 = false) {
    const int vfa1 = 256 * T[0] * T[1], vfa2 = vfa1 + 256 * T[1] * T[2], vb0 = vfa2 + 256 * T[2] * T[3];
    const int vb1 = vb0 + 16 * T[1], vb2 = vb1 + 16 * T[2], end = vb2 + 16 * T[3];
    if (e < vfa1) return map_frag(n, 0, e, T[0], true, p64);
    if (e < vfa2) return map_frag(n, 1, e - vfa1, T[1], true, p64);
    if (e < vb0) return map_frag(n, 2, e - vfa2, T[2], true, p64);
    if (e < vb1) return e - vb0 < n.L[1] ? n.boff[0] + (e - vb0) : -1;
    if (e < vb2) return e - vb1 < n.L[2] ? n.boff[1] + (e - vb1) : -1;
    if (e < end) return e - vb2 < n.L[3] ? n.boff[2] + (e - vb2) : -1;
    return -1;
}

// natural weight / bias parameter q -> its v-pack slot (the inverse of vmap_at), or -1 for LogStd:
// lets the CG step scatter p' from natural-order registers straight into the fragment LDS
__device__ __forceinline__ int pslot_at(const Net &n, const int (&T)[4], int q) {
    const int vfa[3] = {0, 256 * T[0] * T[1], 256 * (T[0] * T[1] + T[1] * T[2])};
    const int vb0 = 256 * (T[0] * T[1] + T[1] * T[2] + T[2] * T[3]);
    const int vb[3] = {vb0, vb0 + 16 * T[1], vb0 + 16 * (T[1] + T[2])};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const int lo = n.L[i + 1], w = q - n.woff[i], b = q - n.boff[i];
        if (w >= 0 && w < n.L[i] * lo) {
            const int a = w / lo, o = w - a * lo;          // W_i[a][o]: k-tile a >> 4, out-tile o >> 4
            const int lane = (o & 15) + 16 * ((a & 15) >> 2);
            return vfa[i] + (((o >> 4) * T[i] + (a >> 4)) * 64 + lane) * 4 + (a & 3);
        }
        if (b >= 0 && b < lo) return vb[i] + b;
    }
    return -1;
}

// accumulator-order slab position -> natural parameter (or -1): f4 k over
// [W0 tiles (T0 x T1), W1 (T1 x T2), W2 (T2 x T3), B1 (T1), B2 (T2), B3 (T3)], then lane, r.
__device__ __forceinline__ int imap_at(const Net &n, const int (&T)[4], int j) {
    const int k = j >> 8, lane = (j >> 2) & 63, r = j & 3, c = lane & 15, g = lane >> 4;
    int base = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const int nt = T[i] * T[i + 1];
        if (k >= base && k < base + nt) {
            const int at = (k - base) / T[i + 1], bt = (k - base) % T[i + 1];
            const int a = 16 * at + 4 * g + r, b = 16 * bt + c;
            return (a < n.L[i] && b < n.L[i + 1]) ? n.woff[i] + a * n.L[i + 1] + b : -1;
        }
        base += nt;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if (k >= base && k < base + T[i + 1]) {
            const int b = 16 * (k - base) + 4 * g + r;
            return (c == 0 && b < n.L[i + 1]) ? n.boff[i] + b : -1;
        }
        base += T[i + 1];
    }
    return -1;
}

// natural weight/bias parameter q -> accumulator-order slab position (the inverse of imap_at),
// or -1 for LogStd / out of range.  Lets the epilogue issue its cross-block atomics in natural
// order: contiguous, fully populated wave instructions instead of the sparse accumulator rows.
__device__ __forceinline__ int islot_at(const Net &n, const int (&T)[4], int q) {
    int kw[3], kb[3], k = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i) { kw[i] = k; k += T[i] * T[i + 1]; }
#pragma unroll
    for (int i = 0; i < 3; ++i) { kb[i] = k; k += T[i + 1]; }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const int lo = n.L[i + 1], w = q - n.woff[i], b = q - n.boff[i];
        if (w >= 0 && w < n.L[i] * lo) {
            const int a = w / lo, o = w - a * lo;
            return (kw[i] + (a >> 4) * T[i + 1] + (o >> 4)) * 256 + (((a & 15) >> 2) * 16 + (o & 15)) * 4 + (a & 3);
        }
        if (b >= 0 && b < lo) return (kb[i] + (b >> 4)) * 256 + ((b & 15) >> 2) * 64 + (b & 3);
    }
    return -1;
}

__global__ void build_maps_kernel(Net n, Pack pk, int *tmap, int *vmap, int p64) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < pk.tlen) {
        int m = -1;
        for (int i = 0; i < 3; ++i) {
            if (e >= pk.fa[i] && e < pk.fa[i] + 256 * pk.T[i] * pk.T[i + 1])
                m = map_frag(n, i, e - pk.fa[i], pk.T[i], true, p64 != 0);
            if (i > 0 && e >= pk.fb[i] && e < pk.fb[i] + 256 * pk.T[i] * pk.T[i + 1])
                m = map_frag(n, i, e - pk.fb[i], pk.T[i + 1], false, p64 != 0);
            if (e >= pk.bi[i] && e < pk.bi[i] + 16 * pk.T[i + 1]) {
                const int j = e - pk.bi[i];
                m = j < n.L[i + 1] ? n.boff[i] + j : -1;
            }
        }
        tmap[e] = m;
    }
    if (e < pk.vlen) vmap[e] = vmap_at(n, pk.T, e, p64 != 0);
}

// packs are fp32 or (f64 != 0) fp64
__global__ void build_pslot_kernel(Net n, Pack pk, int *ps, int P) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    const int T[4] = {pk.T[0], pk.T[1], pk.T[2], pk.T[3]};
    if (q < P) ps[q] = pslot_at(n, T, q);
}
// natural parameter -> accumulator (slab) position of the tile kernel's epilogue, q < nw
__global__ void build_islot_kernel(Net n, Pack pk, int *is, int nw) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    const int T[4] = {pk.T[0], pk.T[1], pk.T[2], pk.T[3]};
    if (q < nw) is[q] = islot_at(n, T, q);
}

__global__ void gather_pack_kernel(void *dst, const double *src, const int *map, int len, int f64) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < len) {
        const int m = map[e];
        const double v = m >= 0 ? src[m] : 0.0;
        if (f64) reinterpret_cast<double *>(dst)[e] = v;
        else reinterpret_cast<float *>(dst)[e] = (float)v;
    }
}

// slab position -> natural parameter index (or -1) for the fast kernel's accumulator order:
// f4 k over [W0 tiles (T0 x T1), W1 (T1 x T2), W2 (T2 x T3), B1 (T1), B2 (T2), B3 (T3)], then lane, r.
__global__ void build_imap_kernel(Net n, Pack pk, int *imap, int slab) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < slab) imap[j] = imap_at(n, pk.T, j);
}

__global__ void iota_kernel(int *v, int len, int valid) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < len) v[j] = j < valid ? j : -1;
}

__global__ void set_invvar_kernel(void *iv, const double *stdv, int A, int len, int f64) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < len) {
        const double v = j < A ? 1.0 / stdv[j] / stdv[j] : 0.0;
        if (f64) reinterpret_cast<double *>(iv)[j] = v;
        else reinterpret_cast<float *>(iv)[j] = (float)v;
    }
}

// observations fp64 [n][L0] -> [npad][16*T0], zero padded; fp32, or fp64 with the features of
// each 16-block in the fp64 MFMA row order (slot 4g + r holds feature g + 4r)
__global__ void obs_pad_kernel(void *dst, const double *src, int n, int npad, int L0, int ld, int f64) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (long)npad * ld) return;
    const int s = (int)(e / ld), k = (int)(e % ld);
    const int q = k & 15, kf = f64 ? (k - q) + (q >> 2) + 4 * (q & 3) : k;
    const double v = (s < n && kf < L0) ? src[(long)s * L0 + kf] : 0.0;
    if (f64) reinterpret_cast<double *>(dst)[e] = v;
    else reinterpret_cast<float *>(dst)[e] = (float)v;
}

__global__ void to_f32_kernel(float *dst, const double *src, int len) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < len) dst[e] = (float)src[e];
}
// fp64 -> the generic path's element type (esz 4: fp32, 8: a copy)
__global__ void to_elem_kernel(void *dst, const double *src, long len, int f64) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= len) return;
    if (f64) reinterpret_cast<double *>(dst)[e] = src[e];
    else reinterpret_cast<float *>(dst)[e] = (float)src[e];
}


// ---------------------------------------------------------------------------
// The fused FVP kernel, 3 weight layers (NumLayers == 4), MFMA path.
// ---------------------------------------------------------------------------
constexpr int SCR_LD = 20;            // scratch row stride (floats): conflict-free b32 writes

template <int T0, int T1, int T2, int T3>
struct FastCfg {
    // theta pack (floats)
    static constexpr int FA0 = 0;
    static constexpr int FA1 = FA0 + 256 * T0 * T1;
    static constexpr int FA2 = FA1 + 256 * T1 * T2;
    static constexpr int FB1 = FA2 + 256 * T2 * T3;
    static constexpr int FB2 = FB1 + 256 * T1 * T2;
    static constexpr int BI0 = FB2 + 256 * T2 * T3;
    static constexpr int BI1 = BI0 + 16 * T1;
    static constexpr int BI2 = BI1 + 16 * T2;
    static constexpr int IV = BI2 + 16 * T3;
    static constexpr int TLEN = IV + 16 * T3;
    // v pack (floats), placed right after the theta pack in LDS
    static constexpr int VFA0 = 0;
    static constexpr int VFA1 = VFA0 + 256 * T0 * T1;
    static constexpr int VFA2 = VFA1 + 256 * T1 * T2;
    static constexpr int VB0 = VFA2 + 256 * T2 * T3;
    static constexpr int VB1 = VB0 + 16 * T1;
    static constexpr int VB2 = VB1 + 16 * T2;
    static constexpr int VLEN = VB2 + 16 * T3;
    // per-wave transpose scratch: max rows over the three contractions
    static constexpr int R0 = 16 * (T0 + T1), R1 = 16 * (T1 + T2), R2 = 16 * (T2 + T3);
    static constexpr int ROWS = R0 > R1 ? (R0 > R2 ? R0 : R2) : (R1 > R2 ? R1 : R2);
    static constexpr int SCR = ROWS * 20;             // scr_off: 20 floats per row either way
    // accumulator registers per lane; the block's partial sums are written in this
    // "accumulator order" (f4 k, lane, r) -- SLAB floats per block, mapped back to
    // natural parameter order by the reduce kernel (imap)
    static constexpr int NACC = 4 * (T0 * T1 + T1 * T2 + T2 * T3 + T1 + T2 + T3);
    static constexpr int SLAB = NACC * 64;
    // small nets: weights live in registers and 16 waves per block keep <= 1 tile per wave
    static constexpr bool REGW = T0 * T1 + T1 * T2 + T2 * T3 <= 3;
    // 12 waves (3 per SIMD) for the small nets: ~1 tile per wave at N = 50k, balanced SIMDs
    static constexpr int WAVES = 8;
    // tiles per trip of the cached-forward kernels (MODE 2 / 3).  Round 6 measured two
    // tiles per trip, their MFMA chains interleaved instruction by instruction and every sum in the same order
    // (bit-identical): slower at every size -- CG-iteration kernel 169.1 -> 171.9 us at 4M, 24.4 -> 26.0 us at
    // 500k, 8.8 -> 9.7 us at 50k (profiles/r06_nt2_ab.log) -- so one tile per trip stays; the tile step
    // keeps the NT-generic form
    static constexpr int NT_YC = 1;
    static constexpr int THREADS = 64 * WAVES;
    static constexpr int PMAX = 256 * (T0 * T1 + T1 * T2 + T2 * T3) + 16 * (T1 + T2 + 2 * T3);
    // tile scratch; also stages the fp64 direction of the fused CG update
    static constexpr int SCRATCH = (WAVES * NT_YC * SCR > 2 * PMAX) ? WAVES * NT_YC * SCR : 2 * PMAX;
    static constexpr int MAIN_BYTES = 4 * (TLEN + VLEN + SCRATCH);
    static constexpr int CAP = MAIN_BYTES > 131072 ? MAIN_BYTES : 131072;
    // waves combined per epilogue round (largest divisor of WAVES whose dumps fit)
    static constexpr int rw_pick(int w) {
        return w < 1 ? 1 : ((WAVES % w == 0 && w * SLAB * 4 <= CAP) ? w : rw_pick(w - 1));
    }
    static constexpr int RW = rw_pick(WAVES);
    static constexpr int EPT = (SLAB / 4 + THREADS - 1) / THREADS;   // f4 slices per thread in the combine
    // fused CG update: natural P-vector elements per thread (upper bound from the padded shape)
    static constexpr int EMAX = (PMAX + THREADS - 1) / THREADS;
    static constexpr int VEMAX = (VLEN + THREADS - 1) / THREADS;
    static constexpr int EMAX_REPLICAS = 4;        // atomic-replica reduction only for EMAX <= this
    static_assert(NT_YC == 1 || NT_YC == 2, "NT");
    static_assert(WAVES % RW == 0, "RW");
    static int lds_bytes() {
        const int b = 4 * RW * SLAB;
        return MAIN_BYTES > b ? MAIN_BYTES : b;
    }
};

// sum over the 16 lanes of a DPP row (the 16 sample columns of a D tile), all lanes get it
__device__ __forceinline__ float rowsum16(float v) {
    int x = __float_as_int(v);
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false));   // quad_perm xor 1
    x = __float_as_int(v);
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false));   // quad_perm xor 2
    x = __float_as_int(v);
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x124, 0xF, 0xF, false));  // row_ror 4
    x = __float_as_int(v);
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x128, 0xF, 0xF, false));  // row_ror 8
    return v;
}

// sum of one value over the four 16-lane rows of a wave (gfx950 v_permlane32_swap, v_permlane16_swap):
// (row 0 + row 2) + (row 1 + row 3), the same bits in every lane
__device__ __forceinline__ float rowgroup_sum(float v) {
    const auto h = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    const float t = __uint_as_float(h[0]) + __uint_as_float(h[1]);
    const auto q = __builtin_amdgcn_permlane16_swap(__float_as_uint(t), __float_as_uint(t), false, false);
    return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}
// rowgroup_sum of four values at once, transposed: the half-wave swap pairs values 0/1 and 2/3 and the
// row swap pairs the two results, so one swap + one add serves two values (row g of t then holds value
// {0, 2, 1, 3}[g] as (row 0 + row 2) + (row 1 + row 3) -- rowgroup_sum's association, the same bits);
// three more swaps broadcast the four totals back to every row.  12 instructions instead of ~24.
__device__ __forceinline__ f4 rowgroup_sum4(f4 v) {
    const auto p01 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[0]), __float_as_uint(v[1]), false, false);
    const auto p23 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[2]), __float_as_uint(v[3]), false, false);
    const float s01 = __uint_as_float(p01[0]) + __uint_as_float(p01[1]);   // rows: v0, v0, v1, v1 (half sums)
    const float s23 = __uint_as_float(p23[0]) + __uint_as_float(p23[1]);   // rows: v2, v2, v3, v3
    const auto q = __builtin_amdgcn_permlane16_swap(__float_as_uint(s01), __float_as_uint(s23), false, false);
    const float t = __uint_as_float(q[0]) + __uint_as_float(q[1]);         // rows: v0, v2, v1, v3
    const auto h = __builtin_amdgcn_permlane32_swap(__float_as_uint(t), __float_as_uint(t), false, false);
    const auto b02 = __builtin_amdgcn_permlane16_swap(h[0], h[0], false, false);   // rows 0, 1 of t
    const auto b13 = __builtin_amdgcn_permlane16_swap(h[1], h[1], false, false);   // rows 2, 3 of t
    f4 r;
    r[0] = __uint_as_float(b02[0]);
    r[1] = __uint_as_float(b13[0]);
    r[2] = __uint_as_float(b02[1]);
    r[3] = __uint_as_float(b13[1]);
    return r;
}

// Transpose scratch of fvp_mlp3_kernel: scr_put writes lane (c, g)'s accumulator rows 4g + r of
// column c (ds_write_b32), scr_get reads row c's columns 4g .. 4g + 3 (ds_read_b128).  Layout
// (TRPO_SCR_SWZ, round 2): 16 floats per row, 16 floats of gap after every 4 rows, and the 4-float
// chunk index XORed with s(q) = {0, 3, 2, 1}[q], q = (row / 4) mod 4 (rows start at multiples of
// 16).  With gfx950's lane groups (MI355X_MICROARCH.md §LDS): a ds_write_b32 half-wave writes rows
// r and r + 4, whose bases differ by 80 floats = 16 banks mod 32, into disjoint bank halves; the
// ds_read_b128 groups ({0-3,12-15,20-27} and the three others) cover every bank exactly once.  The
// round-1 row stride of 20 floats left 3 two-way conflicts per read group (42 % of the kernel's LDS
// cycles were conflict cycles).  Same footprint: 20 floats per row.
// the tile loop's streamed inputs (observations, forward cache)
__device__ __forceinline__ f4 stream_ld(const f4 *p) {
    return *p;
}

__device__ __forceinline__ int scr_off(int row, int chunk) {
    const int q = (row >> 2) & 3;
    return row * 16 + (row >> 2) * 16 + ((chunk ^ ((4 - q) & 3)) << 2);
}
// TRPO_SCR_XT (round 4): the tile is stored as it is held -- ONE ds_write_b128 of the lane's D-layout
// registers at V index lane + lane / 16 (a 4-float pad after every 16 lanes; 272 of the 320 floats a
// tile slot has) -- and read transposed: lane (c, g) takes feature c of samples 4g .. 4g + 3 from
// floats 4 (4g + 17 (c / 4)) + c % 4 + 4s of the slot (two ds_read2_b32; banks 16g + 4 (c / 4) +
// c % 4 + 4s mod 64, distinct over the 64 lanes).  hipcc issues the reads as four ds_read_b32 here (not
// ds_read2_b32: the constant part of the slot address exceeds its 8-bit offsets), so the count stays 5.
__device__ __forceinline__ void scr_put(float *scr, int row0, f4 t, int c, int g) {
    reinterpret_cast<f4 *>(scr)[(row0 >> 4) * 68 + c + 17 * g] = t;
}
__device__ __forceinline__ f4 scr_get(const float *scr, int row0, int c, int g) {
    const float *p = scr + (row0 >> 4) * 272 + 4 * (4 * g + 17 * (c >> 2)) + (c & 3);
    f4 r;
    r[0] = p[0];
    r[1] = p[4];
    r[2] = p[8];
    r[3] = p[12];
    return r;
}

// ACT >= 0: activations of layers 1..3 fixed at compile time (a1 | a2 << 2 | a3 << 4);
// ACT == -1: read from net.act at run time (wave-uniform branches).
// MODE 0: Fisher-vector product (R-forward + Pearlmutter backward, optionally fused with the
// CG step).  MODE 1: policy gradient of TRPO_Update (plain forward, output seed
// Adv (Action - Mean) / sigma^2, the same backward and contractions; no R chains).
// MODE 2: MODE 0 with the forward activations y1, y2 (y3) read from the cache a MODE 0 launch
// wrote for the same theta and observations: theta is fixed across the FVPs of a CG solve, so
// only the R chains (linear in v) are recomputed -- 40 instead of 48 MFMAs and no tanh per tile.
// MODE 3: MODE 2 as launched inside the CG graph (K_1 ..): identical code under its own name, so a
// kernel trace separates the standalone FVP kernel from the fused CG-iteration kernels.
// QB (MODE 3 only): basis vectors of the residual reorthogonalisation loaded in the prologue's single
// load round (slots >= A.nq read zeros); QB = 0 with an update: the streaming form (qdots_stage1).
// The leading scalar arguments duplicate the IterArgs fields the CG step's first load round needs
// (acc_in, p_in, r_in, x, pslot, the basis; Ps | R_in << 20 | nq << 26 -- 13 dwords): built with
// -mllvm -amdgpu-kernarg-preload-count (14 SGPRs at most besides the kernarg pointer) they arrive in
// SGPRs at wave start, so those loads issue without waiting for a scalar load of the kernarg segment
// (a byval aggregate is never preloaded).
// NO (narrow output layer, T3 == 1 and at most NO <= 4 outputs): the output layer's
// forward / R-forward run on v_mfma_f32_4x4x1_16b_f32 -- lane (c, g) is block 4g + c / 4, column
// c & 3: instruction s multiplies hidden neuron 4g + s of sample c by the weight row of output i in
// register i, and a two-step permlane sum over the lane groups g completes the sum over the hidden
// neurons, leaving outputs 0..3 of sample c in registers 0..3 of EVERY lane group (not only g = 0);
// G2 = W2 G3 and the RGW2 / B3 contractions then run on the VALU (per-lane partials over the
// lane's sample column, summed over the 16 columns once in the epilogue).  With 16x16x4 MFMAs the
// 3-wide output layer took 16 of the 40 MFMAs per tile, 13/16 of their products padding.
// NO encoding: outputs handled (NO & 7, <= 4) | 8 when RGW2 / B3 stay on the 16x16x4 contraction
// ("lite": no per-lane partials, so no 16-column reduction in the epilogue -- the better choice when a
// wave runs only a few tiles; the VALU partials win once the tile loop dominates, bench C4_sweep)
constexpr int NO_MFMA_RGW2 = 8;
template <int T0, int T1, int T2, int T3, int ACT, int MODE, int QB = 0, int NO = 0>
__global__ void __launch_bounds__((64 * FastCfg<T0, T1, T2, T3>::WAVES))
fvp_mlp3_kernel(const double *__restrict__ k_acc, const double *__restrict__ k_p, const double *__restrict__ k_r,
                const double *__restrict__ k_x, const int *__restrict__ k_pslot, const void *k_q, int k_meta,
                IterArgs A, Net net) {
    constexpr bool FV = MODE != 1;
    constexpr bool YC = MODE == 2 || MODE == 3;     // forward activations from the cache
    constexpr int NYC = T1 + T2 + T3;               // cached f4 per lane per tile
    using C = FastCfg<T0, T1, T2, T3>;
    constexpr int NT = YC ? C::NT_YC : 1;           // tiles per trip
    // the cache only for the register-resident small nets: on the wide shapes its extra registers
    // push the kernel into scratch spills (and those runs were not bitwise reproducible)
    static_assert(!YC || C::REGW, "forward cache only for the small-net kernels");
    extern __shared__ __attribute__((aligned(16))) float lds[];
    __shared__ double sh64[(5 + QB) * 4 * C::WAVES];      // 5 + QB DPP block sums, 4 rows per wave
    // streaming basis dots of a MODE 0 update: the tile scratch, unused until the tile loop's barrier
    double *shq = reinterpret_cast<double *>(lds + C::TLEN + C::VLEN);
    float *qf = reinterpret_cast<float *>(A.q);                     // fp32 reorthogonalisation basis
    const float *qfz = reinterpret_cast<const float *>(A.qz);
    const int kPs = k_meta & 0xFFFFF, kR = (k_meta >> 20) & 63, knq = (k_meta >> 26) & 63;
    const float *kq = reinterpret_cast<const float *>(k_q);
    static_assert(C::SCRATCH >= 2 * QCAP * 4 * C::WAVES, "basis-dot scratch");
    float *tw = lds;                                   // theta pack
    float *vw = lds + C::TLEN;                         // v pack (fragment order, fp32)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int c = lane & 15, g = lane >> 4;
    float *scr = lds + C::TLEN + C::VLEN + wave * C::NT_YC * C::SCR;
    const int nwaves = gridDim.x * C::WAVES;
    const int ntiles = A.ntiles, n = A.n;
    const f4 *obs4 = reinterpret_cast<const f4 *>(A.obs4);

    // ---- prologue: ONE round of global loads (flags, theta pack, [v pack | CG state], first tile) ----
    // MODE 3 is always a CG update (compile time: no run-time mode branches around its loads)
    constexpr bool CGK = MODE == 3;
    const bool upd = CGK || (MODE == 0 && A.update != 0);
    const bool ini = !CGK && MODE == 0 && !upd && A.init != 0;
    const bool vnat = !CGK && !upd && !ini && A.v_nat != nullptr;   // plain FVP of a natural-order direction
    constexpr int NT4 = C::TLEN / 4, NALL = CGK ? NT4 : (C::TLEN + C::VLEN) / 4;   // MODE 3: no v pack
    constexpr int PER = (NALL + C::THREADS - 1) / C::THREADS;
    const int skipv = *A.skip;
    // NOTE: every prologue load is unconditional (indices clamped, values selected after):
    // a load guarded by a run-time condition makes hipcc branch around it and drain vmcnt,
    // which serialises the round trips (cdna_hip_programming.md §5 trap (c)).
    f4 st[PER];
    // the wave's tile index is wave-uniform: kept in an SGPR (readfirstlane), the tile loop's
    // bookkeeping, bound test and input addresses are scalar work, not VALU
    int tile = __builtin_amdgcn_readfirstlane(blockIdx.x * C::WAVES + wave);
    // input slots of the tile loop (NT tiles each): slot 0 is the first trip's; the cached-forward kernels
    // stream the later trips through a ring of two slots, the others through one slot and a copy
    constexpr bool RING = YC;
    constexpr int PFU = RING ? 2 : 1;
    f4 xb[PFU][NT][T0];
    [[maybe_unused]] f4 yb[PFU][NT][YC ? NYC : 1];
    f4(&xn)[T0] = xb[0][0];
    const f4 *yc4 = reinterpret_cast<const f4 *>(A.yc);
    const int a3c = ACT >= 0 ? ((ACT >> 4) & 3) : net.act[3];
    // the loads that do not depend on the previous kernel: theta [+ v] pack and the first tile.
    // MODE 3 issues them after the CG state, so the CG step's operands arrive first (loads return
    // in issue order) and these land while the step computes.
    auto load_static = [&]() {
        const f4 *tp4 = reinterpret_cast<const f4 *>(A.tpack);
        const f4 *vp4 = reinterpret_cast<const f4 *>(A.vpack);
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int e = min(tid + k * C::THREADS, NALL - 1);
            st[k] = e < NT4 ? tp4[e] : vp4[e - NT4];
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int tl = max(0, min(tile + t * nwaves, ntiles - 1));
#pragma unroll
            for (int kt = 0; kt < T0; ++kt) xb[0][t][kt] = obs4[(long)(tl * 16 + c) * (4 * T0) + kt * 4 + g];
            if constexpr (YC) {
#pragma unroll
                for (int k = 0; k < T1 + T2; ++k) yb[0][t][k] = yc4[((long)tl * NYC + k) * 64 + lane];
                if (act_needs_y(a3c))
#pragma unroll
                    for (int k = T1 + T2; k < NYC; ++k) yb[0][t][k] = yc4[((long)tl * NYC + k) * 64 + lane];
            }
        }
    };
    if constexpr (!CGK) load_static();
    constexpr int Tc[4] = {T0, T1, T2, T3};
    // CG-step element layout: adjacent pairs (one 16-byte load per vector per thread) where two
    // elements per thread cover P, else the strided layout (elem_of)
    constexpr bool PAIR = C::EMAX == 2;
    // CG state for the fused update (src/TRPO_CG.c:77-103), loaded in the same round
    double pv[C::EMAX], rv[C::EMAX], zv[C::EMAX], xv[C::EMAX];
    int vm[C::VEMAX], ps[C::EMAX];
    CgSt sin = {0.0, 0.0, 0, 0};
    double cn = 1.0, clam = 0.0, cth = 0.0;
    int cmax = 0;
    if (upd) {
        #pragma clang fp contract(off)   // explicit rounding: MODE 0 and MODE 3 give the same bits
        sin = *A.st_in;
        cn = A.ctl->n_total;
        clam = A.ctl->damping;
        cth = A.ctl->resth;
        cmax = A.ctl->maxiter;
        const double *xs = blockIdx.x == 0 ? A.x : A.p_in;    // only block 0 needs x
        if constexpr (PAIR) {
            // replicas summed in replica order as below; rows of stride Ps, pairs 16-byte aligned
            // (the preloaded scalar arguments: no wait for the kernarg segment before these loads)
            const double *xk = blockIdx.x == 0 ? k_x : k_p;
            // waves whose first pair lies beyond Ps hold no CG element (armDOF_0: waves 5-7): they skip
            // the state loads in a wave-uniform scalar branch and keep zeros
            const bool holds = 128 * __builtin_amdgcn_readfirstlane(wave) < kPs;
            double2 p2 = {0.0, 0.0}, r2 = {0.0, 0.0}, x2 = {0.0, 0.0};
            double2 za[RMAX];
#pragma unroll
            for (int k = 0; k < RMAX; ++k) za[k] = make_double2(0.0, 0.0);
            int2 m2 = make_int2(-1, -1);
            if (holds) {
                p2 = pair_at(k_p, 0, kPs);
                r2 = pair_at(k_r, 0, kPs);
                x2 = pair_at(xk, 0, kPs);
#pragma unroll
                for (int k = 0; k < RMAX; ++k) za[k] = pair_at(k_acc, min(k, kR - 1), kPs);
                m2 = pair_at(k_pslot, 0, kPs);
            }
            const double p0[2] = {p2.x, p2.y}, r0[2] = {r2.x, r2.y}, x0[2] = {x2.x, x2.y};
            const int mm[2] = {m2.x, m2.y};
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int q = 2 * tid + e;
                const bool in = q < A.P;
                double z = e ? za[0].y : za[0].x;
#pragma unroll
                for (int k = 1; k < RMAX; ++k) z += k < kR ? (e ? za[k].y : za[k].x) : 0.0;
                pv[e] = in ? p0[e] : 0.0;
                rv[e] = in ? r0[e] : 0.0;
                xv[e] = (in && blockIdx.x == 0) ? x0[e] : 0.0;
                zv[e] = q < A.nw ? z : 0.0;
                ps[e] = in ? mm[e] : -1;
            }
        } else {
#pragma unroll
        for (int e = 0; e < C::EMAX; ++e) {
            const int q = tid + e * C::THREADS, qc = min(q, A.P - 1), qz = min(q, A.nw - 1);
            const bool in = q < A.P;
            const double p0 = A.p_in[qc], r0 = A.r_in[qc], x0 = xs[qc];
            double z = 0.0;
            if constexpr (C::EMAX <= C::EMAX_REPLICAS) {
                // up to 8 atomic replicas (small P only: 8 loads per element in flight)
                double za[RMAX];
#pragma unroll
                for (int k = 0; k < RMAX; ++k) za[k] = A.acc_in[(long)min(k, A.R_in - 1) * A.Ps + qz];
                z = za[0];                                // R_in >= 1: no select on the first term
#pragma unroll
                for (int k = 1; k < RMAX; ++k) z += k < A.R_in ? za[k] : 0.0;
            } else {
                z = A.acc_in[qz];                         // slab mode: one reduced vector
            }
            pv[e] = in ? p0 : 0.0;
            rv[e] = in ? r0 : 0.0;
            xv[e] = (in && blockIdx.x == 0) ? x0 : 0.0;
            zv[e] = q < A.nw ? z : 0.0;
        }
#pragma unroll
        for (int e = 0; e < C::EMAX; ++e) {
            const int q = tid + e * C::THREADS, m = A.pslot[min(q, A.P - 1)];
            ps[e] = q < A.P ? m : -1;
        }
        }
#pragma unroll
        for (int e = 0; e < C::VEMAX; ++e) vm[e] = vmap_at(net, Tc, tid + e * C::THREADS);
    } else if (ini) {
#pragma unroll
        for (int e = 0; e < C::EMAX; ++e) {
            const int q = tid + e * C::THREADS;
            const double b0 = A.b_init[min(q, A.P - 1)];
            pv[e] = q < A.P ? b0 : 0.0;
        }
#pragma unroll
        for (int e = 0; e < C::VEMAX; ++e) vm[e] = vmap_at(net, Tc, tid + e * C::THREADS);
#pragma unroll
        for (int e = 0; e < C::EMAX; ++e) {
            const int q = tid + e * C::THREADS, m = A.pslot[min(q, A.P - 1)];
            ps[e] = q < A.P ? m : -1;
        }
    }
    // the reorthogonalisation basis, in the same load round (MODE 3 kernels launched with QB > 0)
    [[maybe_unused]] double qv[QB > 0 ? QB : 1][C::EMAX];
    if constexpr (QB > 0) {
#pragma unroll
        for (int i = 0; i < QB; ++i) {
            if constexpr (PAIR) {
                // QB > 0 implies nq >= 1 (qb_index): the clamped row is a stored basis vector, selected
                // away for the slots >= nq (no zero-line pointer needed); skipped by element-less waves
                float2 v = make_float2(0.0f, 0.0f);
                if (128 * __builtin_amdgcn_readfirstlane(wave) < kPs) v = pair_at(kq, min(i, knq - 1), kPs);
                const bool ok = i < knq;
                qv[i][0] = (ok && 2 * tid < A.P) ? (double)v.x : 0.0;
                qv[i][1] = (ok && 2 * tid + 1 < A.P) ? (double)v.y : 0.0;
            } else {
                qload<C::EMAX, float, PAIR>(qv[i], qf, qfz, A.P, A.Ps, i, upd ? A.nq : 0, C::THREADS);
            }
        }
    }
    if constexpr (CGK) load_static();
    // plain FVP: the direction fragments gathered from v in the same load round
    float vg[C::VEMAX];
    if (vnat) {
#pragma unroll
        for (int e = 0; e < C::VEMAX; ++e) {
            const int m = vmap_at(net, Tc, tid + e * C::THREADS);      // -1 past VLEN
            const double v = A.v_nat[max(m, 0)];
            vg[e] = m >= 0 ? (float)v : 0.0f;
        }
    }
    if (skipv) return;                                 // grid-uniform
    auto stage_static = [&]() {
        f4 *dst = reinterpret_cast<f4 *>(lds);
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int e = tid + k * C::THREADS;
            if (e < NT4 || (e < NALL && !upd && !ini && !vnat)) dst[e] = st[k];
        }
    };
    if constexpr (!CGK) stage_static();               // MODE 3: after the CG step (its loads came last)
    if (vnat) {
#pragma unroll
        for (int e = 0; e < C::VEMAX; ++e) {
            const int ve = tid + e * C::THREADS;
            if (ve < C::VLEN) vw[ve] = vg[e];
        }
    }
    if (ini) {
        #pragma clang fp contract(off)   // explicit rounding: MODE 0 and MODE 3 give the same bits
#pragma unroll
        for (int e = 0; e < C::EMAX; ++e)
            if (ps[e] >= 0) vw[ps[e]] = (float)pv[e];
#pragma unroll
        for (int e = 0; e < C::VEMAX; ++e) {
            const int ve = tid + e * C::THREADS;
            if (ve < C::VLEN && vm[e] < 0) vw[ve] = 0.0f;
        }
        if (blockIdx.x == gridDim.x - 1) {             // block-uniform; the block with the fewest tiles
            double red[1] = {0.0};
#pragma unroll
            for (int e = 0; e < C::EMAX; ++e) red[0] += pv[e] * pv[e];
            block_sums_dpp<1, C::WAVES>(red, sh64);
            const double rr = red[0];
#pragma unroll
            for (int e = 0; e < C::EMAX; ++e) {
                const int q = tid + e * C::THREADS;
                if (q < A.P) {
                    A.p_out[q] = pv[e];
                    A.r_out[q] = pv[e];
                    A.x[q] = 0.0;
                }
            }
            if (A.reorth) qstore<C::EMAX>(qf, A.P, A.Ps, 0, rr, pv, C::THREADS);     // q_0 = b / |b|
            if (tid == 0) {
                A.st_out->rdotr = rr;
                A.st_out->xx = 0.0;
                A.st_out->iter = 0;
                A.hist[0] = rr;
                A.hist[1] = 0.0;
                A.ctl->maxiter = A.init_maxiter;
                A.ctl->resth = A.init_resth;
                A.ctl->rdotr = rr;
                A.ctl->iter = 0;
                A.ctl->orth = 0.0;
                A.ctl->done = (rr < A.init_resth || A.init_maxiter == 0) ? 1 : 0;
            }
        }
    }
    if (upd) {
        #pragma clang fp contract(off)   // explicit rounding: MODE 0 and MODE 3 give the same bits
        // every block runs the identical fp64 CG step (fixed-order sums => bitwise-equal
        // results in all blocks); block 0 publishes the new state
        // ONE block reduction per step: p.z, r.z, z.z, x.p, p.p; then |r'|^2 = |r|^2 - 2a r.z + a^2 z.z
        // and |x'|^2 = |x|^2 + 2a x.p + a^2 p.p in fp64 (algebraically the reference's r.r / x.x)
        // + the basis dots q_i . z of the residual reorthogonalisation (QB of them in registers, or the
        // streaming stage 1 into shq), in the same single barrier
        double red[5 + QB];
#pragma unroll
        for (int k = 0; k < 5 + QB; ++k) red[k] = 0.0;
#pragma unroll
        for (int e = 0; e < C::EMAX; ++e) {
            const int q = elem_of<PAIR>(e, C::THREADS);
            // contraction is off in this block: the fused multiply-adds are spelled out
            zv[e] = __builtin_fma(clam, pv[e], q < A.nw ? zv[e] / cn : 2.0 * pv[e]);
            red[0] = __builtin_fma(pv[e], zv[e], red[0]);
            red[1] = __builtin_fma(rv[e], zv[e], red[1]);
            red[2] = __builtin_fma(zv[e], zv[e], red[2]);
            red[3] = __builtin_fma(xv[e], pv[e], red[3]);
            red[4] = __builtin_fma(pv[e], pv[e], red[4]);
#pragma unroll
            for (int i = 0; i < QB; ++i) red[5 + i] = __builtin_fma(qv[i][e], zv[e], red[5 + i]);
        }
        if constexpr (QB == 0) {
            if (A.reorth && A.nq > 0) qdots_stage1<C::EMAX, float, PAIR>(qf, qfz, A.P, A.Ps, A.nq, zv, C::THREADS, shq);
        }
        block_sums_dpp<5 + QB, C::WAVES>(red, sh64);
        const double alpha = sin.rdotr / red[0];
        // coefficient along the current residual r (unit vector r / |r|): |r| - alpha (r . z) / |r|
        double cs = 0.0, cr = 0.0;
        if (A.reorth && sin.rdotr > 0.0) {
            const double nrm = sqrt(sin.rdotr), cl = nrm - alpha * (red[1] / nrm);
            cs = cl * cl;
            cr = cl / nrm;
        }
#pragma unroll
        for (int e = 0; e < C::EMAX; ++e) {
            const double r0 = rv[e];
            rv[e] = __builtin_fma(-alpha, zv[e], rv[e]);
            rv[e] = __builtin_fma(-cr, r0, rv[e]);
            xv[e] = __builtin_fma(alpha, pv[e], xv[e]);
        }
        if constexpr (QB > 0) {
#pragma unroll
            for (int i = 0; i < QB; ++i) {
                const double c = -alpha * red[5 + i];       // zero for the slots >= nq
                cs += c * c;
#pragma unroll
                for (int e = 0; e < C::EMAX; ++e) rv[e] = __builtin_fma(-c, qv[i][e], rv[e]);
            }
        } else {
            if (A.reorth && A.nq > 0) cs += qcorrect<C::EMAX, float, PAIR>(qf, qfz, A.P, A.Ps, A.nq, C::THREADS, shq, alpha, rv);
        }
        const double nr = sin.rdotr - 2.0 * alpha * red[1] + alpha * alpha * red[2] - cs;
        const double xn2 = sin.xx + 2.0 * alpha * red[3] + alpha * alpha * red[4];
        const double beta = nr / sin.rdotr;
#pragma unroll
        for (int e = 0; e < C::EMAX; ++e) {
            const int q = elem_of<PAIR>(e, C::THREADS);
            pv[e] = __builtin_fma(beta, pv[e], rv[e]);
            if (q < A.P && blockIdx.x == 0) {
                A.p_out[q] = pv[e];
                A.r_out[q] = rv[e];
                A.x[q] = xv[e];
            }
        }
        const int it = sin.iter + 1;
        const int done = (nr < cth || it >= cmax) ? 1 : 0;
        if (blockIdx.x == 0 && A.reorth) qstore<C::EMAX, float, PAIR>(qf, A.P, A.Ps, it, nr, rv, C::THREADS);
        if (blockIdx.x == 0 && tid == 0) {
            A.st_out->rdotr = nr;
            A.st_out->xx = xn2;
            A.st_out->iter = it;
            A.hist[2 * it] = nr;
            A.hist[2 * it + 1] = sqrt(xn2);
            A.ctl->rdotr = nr;
            A.ctl->iter = it;
            A.ctl->done = done;
            note_orth(&A.ctl->orth, cs, nr);
            if (it <= CG_AMAX) A.ctl->alpha[it - 1] = alpha;
        }
        if (done) return;                              // block-uniform (identical in every block)
        // p' straight into the fragment LDS: natural element q -> its pack slot (an LDS scatter),
        // the padding slots zeroed by their owners -- disjoint writes, so no staging barrier
#pragma unroll
        for (int e = 0; e < C::EMAX; ++e)
            if (ps[e] >= 0) vw[ps[e]] = (float)pv[e];
#pragma unroll
        for (int e = 0; e < C::VEMAX; ++e) {
            const int ve = tid + e * C::THREADS;
            if (ve < C::VLEN && vm[e] < 0) vw[ve] = 0.0f;
        }
    }
    if constexpr (CGK) stage_static();
    __syncthreads();
    // the epilogue's natural -> accumulator positions (a table built at context creation: islot_at's
    // integer divisions cost ~0.3 us per launch on the epilogue's critical path); loaded now, used
    // after the tile loop, so the load's latency hides behind the tiles
    [[maybe_unused]] int jslot[C::EMAX];
    if constexpr (C::RW == C::WAVES) {
        if (A.islot) {
#pragma unroll
            for (int e = 0; e < C::EMAX; ++e) jslot[e] = A.islot[min(tid + e * C::THREADS, A.nw - 1)];
        }
    }
    [[maybe_unused]] bool first_tile = true;

    const int a1 = ACT >= 0 ? (ACT & 3) : net.act[1];
    const int a2 = ACT >= 0 ? ((ACT >> 2) & 3) : net.act[2];
    const int a3 = ACT >= 0 ? ((ACT >> 4) & 3) : net.act[3];
    const bool y3_needed = act_needs_y(a3);
    f4 *ycs = (MODE == 0 && C::REGW) ? reinterpret_cast<f4 *>(A.yc) : nullptr;   // cache writer
    const f4 *TW = reinterpret_cast<const f4 *>(tw);
    const f4 *VW = reinterpret_cast<const f4 *>(vw);

    const f4 zero4 = {0.f, 0.f, 0.f, 0.f};
    // small nets: every fragment held in registers across the tile loop (no LDS on the chain)
    f4 rFA0 = zero4, rVFA0 = zero4, rFA1 = zero4, rVFA1 = zero4, rFA2 = zero4, rVFA2 = zero4, rFB1 = zero4,
       rFB2 = zero4;
    if constexpr (C::REGW) {
        rFA0 = TW[C::FA0 / 4 + lane];
        rVFA0 = VW[C::VFA0 / 4 + lane];
        rFA1 = TW[C::FA1 / 4 + lane];
        rVFA1 = VW[C::VFA1 / 4 + lane];
        rFA2 = TW[C::FA2 / 4 + lane];
        rVFA2 = VW[C::VFA2 / 4 + lane];
        rFB1 = TW[C::FB1 / 4 + lane];
        rFB2 = TW[C::FB2 / 4 + lane];
    }
#define WLD(REG, EXPR) (C::REGW ? (REG) : (EXPR))
    constexpr int NOUT = NO & 7;                            // outputs of the narrow layer (0: off)
    static_assert(NO == 0 || (T3 == 1 && NOUT >= 1 && NOUT <= 4), "narrow output layer");
    constexpr int NOA = NOUT ? NOUT : 1;
    constexpr bool NOV = NOUT && !(NO & NO_MFMA_RGW2);      // RGW2 / B3 on the VALU
    [[maybe_unused]] f4 nFA2[T2], nVFA2[T2], w2n[T2][4];    // NO: 4x4 A operands, W2[16kt + 4g + r][0..3]
    [[maybe_unused]] f4 nb2 = zero4, nvb2 = zero4, niv = zero4;
    [[maybe_unused]] float acc2[T2][4][NOA], sb3n[NOA];    // NO: per-lane RGW2 / B3 partials
    if constexpr (NO) {
        const int lp = (c & 3) + 16 * g;                     // FA2 lane holding W2[16kt + 4g + s][c & 3]
#pragma unroll
        for (int kt = 0; kt < T2; ++kt) {
            nFA2[kt] = TW[C::FA2 / 4 + kt * 64 + lp];
            nVFA2[kt] = FV ? VW[C::VFA2 / 4 + kt * 64 + lp] : zero4;
#pragma unroll
            for (int r = 0; r < 4; ++r) w2n[kt][r] = TW[C::FB2 / 4 + kt * 64 + 4 * g + r];   // FB2 lane 4g + r
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int o = 0; o < NOA; ++o) acc2[kt][r][o] = 0.0f;
        }
        nb2 = g == 0 ? TW[C::BI2 / 4] : zero4;               // biases enter once: row group 0 only
        nvb2 = (FV && g == 0) ? VW[C::VB2 / 4] : zero4;
        niv = TW[C::IV / 4];
#pragma unroll
        for (int o = 0; o < NOA; ++o) sb3n[o] = 0.0f;
    }
    f4 accW0[T0][T1], accW1[T1][T2], accW2[T2][T3];
    f4 sB1[T1], sB2[T2], sB3[T3];
#pragma unroll
    for (int a = 0; a < T0; ++a)
#pragma unroll
        for (int b = 0; b < T1; ++b) accW0[a][b] = zero4;
#pragma unroll
    for (int a = 0; a < T1; ++a)
#pragma unroll
        for (int b = 0; b < T2; ++b) accW1[a][b] = zero4;
#pragma unroll
    for (int a = 0; a < T2; ++a)
#pragma unroll
        for (int b = 0; b < T3; ++b) accW2[a][b] = zero4;
#pragma unroll
    for (int a = 0; a < T1; ++a) sB1[a] = zero4;
#pragma unroll
    for (int a = 0; a < T2; ++a) sB2[a] = zero4;
#pragma unroll
    for (int a = 0; a < T3; ++a) sB3[a] = zero4;

    // NT independent tiles per loop trip, their chains interleaved instruction by instruction (the t loops
    // innermost).  Every accumulator still receives the tiles in the order one tile per trip gives (tile
    // t of a trip before tile t + 1, each tile's products in the same order), so the sums are bit-identical.
    [[maybe_unused]] const int pf_xoff = (c * (4 * T0) + g) * 16, pf_yoff = lane * 16;   // prefetch lane offsets (bytes)
    // one tile (NT tiles) of work: inputs x0, the cached activations ycur, live columns
    auto tile_step = [&](const int tile, const f4 (&x0)[NT][T0], const f4 (&ycur)[NT][YC ? NYC : 1],
                         const bool (&live)[NT]) __attribute__((always_inline)) {
        // ---- layer 0: x1 = W0^T x0 + b0 ; Rx1 = VW0^T x0 + vb0 (Ry0 = 0) ----
        f4 y1[NT][T1], r1[NT][T1];
#pragma unroll
        for (int ot = 0; ot < T1; ++ot) {
            const f4 b0 = TW[C::BI0 / 4 + ot * 4 + g], vb0 = VW[C::VB0 / 4 + ot * 4 + g];
            f4 a[NT], ra[NT];
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                a[t] = b0;
                ra[t] = vb0;
            }
#pragma unroll
            for (int kt = 0; kt < T0; ++kt) {
                const f4 w = WLD(rFA0, TW[C::FA0 / 4 + (ot * T0 + kt) * 64 + lane]);
                const f4 u = FV ? WLD(rVFA0, VW[C::VFA0 / 4 + (ot * T0 + kt) * 64 + lane]) : zero4;
#pragma unroll
                for (int s = 0; s < 4; ++s)
#pragma unroll
                    for (int t = 0; t < NT; ++t) {
                        if constexpr (!YC) a[t] = MFMA(w[s], x0[t][kt][s], a[t]);
                        if constexpr (FV) ra[t] = MFMA(u[s], x0[t][kt][s], ra[t]);
                    }
            }
            if constexpr (YC) {
#pragma unroll
                for (int t = 0; t < NT; ++t) {
                    y1[t][ot] = ycur[t][ot];
                    r1[t][ot] = act_r4(a1, y1[t][ot], ra[t]);
                }
            } else {
#pragma unroll
                for (int t = 0; t < NT; ++t) y1[t][ot] = act_fwd(a1, a[t], ra[t], r1[t][ot]);
                if (ycs) ycs[((long)tile * NYC + ot) * 64 + lane] = y1[0][ot];
            }
        }
        // ---- layer 1 ----
        f4 y2[NT][T2], r2[NT][T2];
#pragma unroll
        for (int ot = 0; ot < T2; ++ot) {
            const f4 b1 = TW[C::BI1 / 4 + ot * 4 + g], vb1 = VW[C::VB1 / 4 + ot * 4 + g];
            f4 a[NT], ra[NT], rb[NT];                     // rb: second R chain, halves the depth
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                a[t] = b1;
                ra[t] = vb1;
                rb[t] = zero4;
            }
#pragma unroll
            for (int kt = 0; kt < T1; ++kt) {
                const f4 w = WLD(rFA1, TW[C::FA1 / 4 + (ot * T1 + kt) * 64 + lane]);
                const f4 u = FV ? WLD(rVFA1, VW[C::VFA1 / 4 + (ot * T1 + kt) * 64 + lane]) : zero4;
#pragma unroll
                for (int s = 0; s < 4; ++s)
#pragma unroll
                    for (int t = 0; t < NT; ++t) {
                        if constexpr (!YC) a[t] = MFMA(w[s], y1[t][kt][s], a[t]);
                        if constexpr (FV) {
                            ra[t] = MFMA(w[s], r1[t][kt][s], ra[t]);
                            rb[t] = MFMA(u[s], y1[t][kt][s], rb[t]);
                        }
                    }
            }
            if constexpr (YC) {
#pragma unroll
                for (int t = 0; t < NT; ++t) {
                    y2[t][ot] = ycur[t][T1 + ot];
                    r2[t][ot] = act_r4(a2, y2[t][ot], ra[t] + rb[t]);
                }
            } else {
#pragma unroll
                for (int t = 0; t < NT; ++t) y2[t][ot] = act_fwd(a2, a[t], ra[t] + rb[t], r2[t][ot]);
                if (ycs) ycs[((long)tile * NYC + T1 + ot) * 64 + lane] = y2[0][ot];
            }
        }
        // ---- layer 2 (output) and G3 = act3'(Ry3 / sigma^2) ----
        f4 g3[NT][T3];
        if constexpr (NO) {
            // narrow: outputs 0..3 of sample c in registers 0..3 of every lane (see the kernel comment)
            f4 a[NT], ra[NT], rb[NT];
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                a[t] = nb2;
                ra[t] = nvb2;
                rb[t] = zero4;
            }
#pragma unroll
            for (int kt = 0; kt < T2; ++kt)
#pragma unroll
                for (int s = 0; s < 4; ++s)
#pragma unroll
                    for (int t = 0; t < NT; ++t) {
                        if (!YC && y3_needed) a[t] = MFMA4(nFA2[kt][s], y2[t][kt][s], a[t]);
                        if constexpr (FV) {
                            ra[t] = MFMA4(nFA2[kt][s], r2[t][kt][s], ra[t]);
                            rb[t] = MFMA4(nVFA2[kt][s], y2[t][kt][s], rb[t]);
                        }
                    }
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const f4 rx = FV ? rowgroup_sum4(ra[t] + rb[t]) : zero4;
                f4 r3, gg, y3;
                if constexpr (YC) {
                    y3 = y3_needed ? ycur[t][T1 + T2] : zero4;
                    r3 = act_r4(a3, y3, rx);
                } else {
                    y3 = act_fwd(a3, y3_needed ? rowgroup_sum4(a[t]) : zero4, rx, r3);
                    if (ycs && y3_needed) ycs[((long)tile * NYC + T1 + T2) * 64 + lane] = y3;
                }
                if constexpr (FV) {
                    gg = act_bwd(a3, y3, r3 * niv);
                } else {
                    const int tt = min(tile + t * nwaves, ntiles - 1);
                    const f4 dm = reinterpret_cast<const f4 *>(A.pg_d4)[(long)(tt * 16 + c) * 4];
                    const float adv = A.pg_adv[tt * 16 + c];
                    gg = act_bwd(a3, y3, (adv * dm) * reinterpret_cast<const f4 *>(A.pg_iv4)[0]);
                }
                g3[t][0] = live[t] ? gg : zero4;
                if constexpr (NOV) {
#pragma unroll
                    for (int o = 0; o < NOA; ++o) sb3n[o] += g3[t][0][o];
                }
            }
        } else
#pragma unroll
        for (int ot = 0; ot < T3; ++ot) {
            const f4 b2 = TW[C::BI2 / 4 + ot * 4 + g], vb2 = VW[C::VB2 / 4 + ot * 4 + g];
            const f4 iv = TW[C::IV / 4 + ot * 4 + g];
            f4 a[NT], ra[NT], rb[NT];
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                a[t] = b2;
                ra[t] = vb2;
                rb[t] = zero4;
            }
#pragma unroll
            for (int kt = 0; kt < T2; ++kt) {
                const f4 w = WLD(rFA2, TW[C::FA2 / 4 + (ot * T2 + kt) * 64 + lane]);
                const f4 u = FV ? WLD(rVFA2, VW[C::VFA2 / 4 + (ot * T2 + kt) * 64 + lane]) : zero4;
#pragma unroll
                for (int s = 0; s < 4; ++s)
#pragma unroll
                    for (int t = 0; t < NT; ++t) {
                        if (!YC && y3_needed) a[t] = MFMA(w[s], y2[t][kt][s], a[t]);
                        if constexpr (FV) {
                            ra[t] = MFMA(w[s], r2[t][kt][s], ra[t]);
                            rb[t] = MFMA(u[s], y2[t][kt][s], rb[t]);
                        }
                    }
            }
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                f4 r3, gg, y3;
                if constexpr (YC) {
                    y3 = y3_needed ? ycur[t][T1 + T2 + ot] : zero4;
                    r3 = act_r4(a3, y3, ra[t] + rb[t]);
                } else {
                    y3 = act_fwd(a3, a[t], ra[t] + rb[t], r3);
                    if (ycs && y3_needed) ycs[((long)tile * NYC + T1 + T2 + ot) * 64 + lane] = y3;
                }
                if constexpr (FV) {
                    gg = act_bwd(a3, y3, r3 * iv);
                } else {
                    // seed of the policy gradient (src/TRPO_Update.c:297-303), lane = (sample c, outputs 4g+r)
                    const int tt = min(tile + t * nwaves, ntiles - 1);
                    const f4 dm = reinterpret_cast<const f4 *>(A.pg_d4)[(long)(tt * 16 + c) * (4 * T3) + ot * 4 + g];
                    const float adv = A.pg_adv[tt * 16 + c];
                    gg = act_bwd(a3, y3, (adv * dm) * reinterpret_cast<const f4 *>(A.pg_iv4)[ot * 4 + g]);
                }
                g3[t][ot] = live[t] ? gg : zero4;
                sB3[ot] += g3[t][ot];
            }
        }
        // ---- contraction RGW2 += Y2 . G3^T (K = 16 samples per tile) ----
        [[maybe_unused]] f4 g3m[NT][T3];                  // G3 in the 16x16x4 layout (rows 4g + r)
        if constexpr (NO && !NOV) {
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                g3m[t][0] = g == 0 ? g3[t][0] : zero4;
                sB3[0] += g3m[t][0];
            }
        }
        if constexpr (NOV) {
            // per lane: hidden 16kt + 4g + r x output o of the lane's own sample column
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int kt = 0; kt < T2; ++kt)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
#pragma unroll
                        for (int o = 0; o < NOA; ++o)
                            acc2[kt][r][o] = fmaf(y2[t][kt][r], g3[t][0][o], acc2[kt][r][o]);
        } else {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            float *sc = scr + t * C::SCR;
#pragma unroll
            for (int i = 0; i < T2; ++i) scr_put(sc, 16 * i, y2[t][i], c, g);
#pragma unroll
            for (int i = 0; i < T3; ++i) scr_put(sc, 16 * (T2 + i), NO ? g3m[t][i] : g3[t][i], c, g);
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const float *sc = scr + t * C::SCR;
            f4 gb[T3];
#pragma unroll
            for (int i = 0; i < T3; ++i) gb[i] = scr_get(sc, 16 * (T2 + i), c, g);
#pragma unroll
            for (int at = 0; at < T2; ++at) {
                const f4 ya = scr_get(sc, 16 * at, c, g);
#pragma unroll
                for (int bt = 0; bt < T3; ++bt)
#pragma unroll
                    for (int s = 0; s < 4; ++s) accW2[at][bt] = MFMA(ya[s], gb[bt][s], accW2[at][bt]);
            }
        }
        }
        // ---- G2 = act2'(W2 G3) ----
        f4 g2[NT][T2];
#pragma unroll
        for (int it = 0; it < T2; ++it) {
            f4 a[NT];
#pragma unroll
            for (int t = 0; t < NT; ++t) a[t] = zero4;
            if constexpr (NO) {
                // the fmaf chain over the outputs a 16x16x4 MFMA forms (its padded rows add zeros)
#pragma unroll
                for (int t = 0; t < NT; ++t)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
#pragma unroll
                        for (int o = 0; o < NOA; ++o) a[t][r] = fmaf(w2n[it][r][o], g3[t][0][o], a[t][r]);
            } else
#pragma unroll
            for (int kt = 0; kt < T3; ++kt) {
                const f4 w = WLD(rFB2, TW[C::FB2 / 4 + (it * T3 + kt) * 64 + lane]);
#pragma unroll
                for (int s = 0; s < 4; ++s)
#pragma unroll
                    for (int t = 0; t < NT; ++t) a[t] = MFMA(w[s], g3[t][kt][s], a[t]);
            }
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                g2[t][it] = act_bwd(a2, y2[t][it], a[t]);
                sB2[it] += g2[t][it];
            }
        }
        // ---- contraction RGW1 += Y1 . G2^T ----
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            float *sc = scr + t * C::SCR;
#pragma unroll
            for (int i = 0; i < T1; ++i) scr_put(sc, 16 * i, y1[t][i], c, g);
#pragma unroll
            for (int i = 0; i < T2; ++i) scr_put(sc, 16 * (T1 + i), g2[t][i], c, g);
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const float *sc = scr + t * C::SCR;
            f4 gb[T2];
#pragma unroll
            for (int i = 0; i < T2; ++i) gb[i] = scr_get(sc, 16 * (T1 + i), c, g);
#pragma unroll
            for (int at = 0; at < T1; ++at) {
                const f4 ya = scr_get(sc, 16 * at, c, g);
#pragma unroll
                for (int bt = 0; bt < T2; ++bt)
#pragma unroll
                    for (int s = 0; s < 4; ++s) accW1[at][bt] = MFMA(ya[s], gb[bt][s], accW1[at][bt]);
            }
        }
        // ---- G1 = act1'(W1 G2) ----
        f4 g1[NT][T1];
#pragma unroll
        for (int it = 0; it < T1; ++it) {
            f4 a[NT];
#pragma unroll
            for (int t = 0; t < NT; ++t) a[t] = zero4;
#pragma unroll
            for (int kt = 0; kt < T2; ++kt) {
                const f4 w = WLD(rFB1, TW[C::FB1 / 4 + (it * T2 + kt) * 64 + lane]);
#pragma unroll
                for (int s = 0; s < 4; ++s)
#pragma unroll
                    for (int t = 0; t < NT; ++t) a[t] = MFMA(w[s], g2[t][kt][s], a[t]);
            }
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                g1[t][it] = act_bwd(a1, y1[t][it], a[t]);
                sB1[it] += g1[t][it];
            }
        }
        // ---- contraction RGW0 += X0 . G1^T ----
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            float *sc = scr + t * C::SCR;
#pragma unroll
            for (int i = 0; i < T0; ++i) scr_put(sc, 16 * i, x0[t][i], c, g);
#pragma unroll
            for (int i = 0; i < T1; ++i) scr_put(sc, 16 * (T0 + i), g1[t][i], c, g);
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const float *sc = scr + t * C::SCR;
            f4 gb[T1];
#pragma unroll
            for (int i = 0; i < T1; ++i) gb[i] = scr_get(sc, 16 * (T0 + i), c, g);
#pragma unroll
            for (int at = 0; at < T0; ++at) {
                const f4 ya = scr_get(sc, 16 * at, c, g);
#pragma unroll
                for (int bt = 0; bt < T1; ++bt)
#pragma unroll
                    for (int s = 0; s < 4; ++s) accW0[at][bt] = MFMA(ya[s], gb[bt][s], accW0[at][bt]);
            }
        }
    };
    if constexpr (RING) {
        // the loop unrolled by the ring size, so every slot index is a compile-time constant: trip j of a
        // round issues the loads of trip j + 1 into slot (j + 1) % 2 at its top (buffer loads off per-trip
        // descriptors, clamped to the last tile) and computes on slot j -- the tile step reads the slot
        // registers the loads landed in, with no copy (round 5: 6 v_mov_b64 per tile less).  A trip is NT
        // tiles: tile + t * nwaves, t < NT (the tile -> wave assignment of one tile per trip).
        while (tile < ntiles) {
#pragma unroll
            for (int j = 0; j < PFU; ++j) {
                if (tile >= ntiles) break;
                const int sl = (j + 1) % PFU;
#pragma unroll
                for (int t = 0; t < NT; ++t) {
                    const int tn = min(tile + (NT + t) * nwaves, ntiles - 1);
                    const auto rx = __builtin_amdgcn_make_buffer_rsrc((void *)(obs4 + (long)tn * (16 * 4 * T0)), 0,
                                                                      16 * 64 * T0, 0x00020000);
#pragma unroll
                    for (int kt = 0; kt < T0; ++kt)
                        xb[sl][t][kt] =
                            __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rx, pf_xoff + kt * 64, 0, 0));
                    const auto ry = __builtin_amdgcn_make_buffer_rsrc((void *)(yc4 + (long)tn * (NYC * 64)), 0,
                                                                      NYC * 1024, 0x00020000);
#pragma unroll
                    for (int k = 0; k < T1 + T2; ++k)
                        yb[sl][t][k] =
                            __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(ry, pf_yoff + k * 1024, 0, 0));
                    if (y3_needed)
#pragma unroll
                        for (int k = T1 + T2; k < NYC; ++k)
                            yb[sl][t][k] = __builtin_bit_cast(
                                f4, __builtin_amdgcn_raw_buffer_load_b128(ry, pf_yoff + k * 1024, 0, 0));
                }
                // keep the prefetch at the top of the trip: left to itself hipcc sinks the loads toward
                // their use (4M: 171.0 -> 186.7 us without this, profiles/r05_pf_pin_ab.log)
                __builtin_amdgcn_sched_barrier(0);
                bool live[NT];
#pragma unroll
                for (int t = 0; t < NT; ++t) live[t] = (tile + t * nwaves) * 16 + c < n;
                tile_step(tile, xb[j], yb[j], live);
                tile += NT * nwaves;
            }
        }
    } else {
        static_assert(NT == 1, "one tile per trip outside the cached-forward ring");
        for (; tile < ntiles; tile += nwaves) {
            // input tile: lane holds features 16kt+4g..+3 of its sample (D-layout rows)
            f4 x0[1][T0];
            const f4 ycur[1][1] = {{zero4}};
            const bool live[1] = {tile * 16 + c < n};
#pragma unroll
            for (int kt = 0; kt < T0; ++kt) x0[0][kt] = xn[kt];
            {   // unconditional (clamped) prefetch of the next trip's tile: buffer loads off a per-trip
                // descriptor of the tile's records (the wave-uniform part of the address is SALU work, the
                // lane offsets loop-invariant)
                const int tn = min(tile + nwaves, ntiles - 1);
                const auto rx = __builtin_amdgcn_make_buffer_rsrc((void *)(obs4 + (long)tn * (16 * 4 * T0)), 0,
                                                                  16 * 64 * T0, 0x00020000);
#pragma unroll
                for (int kt = 0; kt < T0; ++kt)
                    xn[kt] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rx, pf_xoff + kt * 64, 0, 0));
                // the prefetch stays at the top of the trip (left to itself the scheduler sinks it to the
                // loop latch, where the x0 = xn copy then waits out a full memory round trip)
                __builtin_amdgcn_sched_barrier(0);
            }
            tile_step(tile, x0, ycur, live);
        }
    }

    // ---- epilogue: bias partials summed over the 16 sample columns (DPP), then the
    //      block's 8 wave copies combined in LDS in a fixed order, all threads writing ----
#pragma unroll
    for (int a = 0; a < T1; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) sB1[a][r] = rowsum16(sB1[a][r]);
#pragma unroll
    for (int a = 0; a < T2; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) sB2[a][r] = rowsum16(sB2[a][r]);
    if constexpr (NOV) {
        // the per-lane partials summed over the 16 sample columns, then laid out as the 16x16x4
        // contraction leaves them: RGW2 lane (c, g) register r = hidden 16kt + 4g + r x output c,
        // B3 lane (c, g) register r = output 4g + r (row group 0 only)
#pragma unroll
        for (int o = 0; o < NOA; ++o) sb3n[o] = rowsum16(sb3n[o]);
#pragma unroll
        for (int kt = 0; kt < T2; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float v = 0.0f;
#pragma unroll
                for (int o = 0; o < NOA; ++o) {
                    const float t = rowsum16(acc2[kt][r][o]);
                    v = c == o ? t : v;
                }
                accW2[kt][0][r] = v;
            }
#pragma unroll
        for (int r = 0; r < 4; ++r) sB3[0][r] = (g == 0 && r < NOA) ? sb3n[r < NOA ? r : 0] : 0.0f;
    } else {
#pragma unroll
    for (int a = 0; a < T3; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) sB3[a][r] = rowsum16(sB3[a][r]);
    }
    f4 acc[C::NACC / 4];
    {
        int k = 0;
#pragma unroll
        for (int a = 0; a < T0; ++a)
#pragma unroll
            for (int b = 0; b < T1; ++b) acc[k++] = accW0[a][b];
#pragma unroll
        for (int a = 0; a < T1; ++a)
#pragma unroll
            for (int b = 0; b < T2; ++b) acc[k++] = accW1[a][b];
#pragma unroll
        for (int a = 0; a < T2; ++a)
#pragma unroll
            for (int b = 0; b < T3; ++b) acc[k++] = accW2[a][b];
#pragma unroll
        for (int a = 0; a < T1; ++a) acc[k++] = sB1[a];
#pragma unroll
        for (int a = 0; a < T2; ++a) acc[k++] = sB2[a];
#pragma unroll
        for (int a = 0; a < T3; ++a) acc[k++] = sB3[a];
    }
    f4 *red = reinterpret_cast<f4 *>(lds);
    if constexpr (C::RW == C::WAVES) {
        if (A.acc_out) {
            // all wave dumps fit at once: each thread sums its natural parameters straight from
            // the dumps (fixed wave order, as below) and adds them with contiguous fp64 atomics
            __syncthreads();
#pragma unroll
            for (int k = 0; k < C::NACC / 4; ++k) red[wave * (C::SLAB / 4) + k * 64 + lane] = acc[k];
            __syncthreads();
            double *dst = A.acc_out + (long)(blockIdx.x % A.R_out) * A.Ps;
#pragma unroll
            for (int e = 0; e < C::EMAX; ++e) {
                const int q = tid + e * C::THREADS;
                if (q < A.nw) {
                    const int j = A.islot ? jslot[e] : islot_at(net, Tc, q);
                    float t = 0.0f;
#pragma unroll
                    for (int w = 0; w < C::WAVES; ++w) t += lds[w * C::SLAB + j];
                    unsafeAtomicAdd(dst + q, (double)t);
                }
            }
            if (blockIdx.x == 0)
                for (int e = tid; e < A.zero_len; e += C::THREADS) A.acc_zero[e] = 0.0;
            return;
        }
    }
    f4 part[C::EPT];
#pragma unroll
    for (int j = 0; j < C::EPT; ++j) part[j] = zero4;
#pragma unroll
    for (int w0 = 0; w0 < C::WAVES; w0 += C::RW) {
        __syncthreads();
        if (wave >= w0 && wave < w0 + C::RW) {
#pragma unroll
            for (int k = 0; k < C::NACC / 4; ++k) red[(wave - w0) * (C::SLAB / 4) + k * 64 + lane] = acc[k];
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < C::EPT; ++j) {
            const int e = tid + j * C::THREADS;
            if (e < C::SLAB / 4) {
#pragma unroll
                for (int w = 0; w < C::RW; ++w) part[j] += red[w * (C::SLAB / 4) + e];
            }
        }
    }
    if (A.acc_out) {
        // cross-block sum by fp64 atomics into R replicas: the fp32 block partials are added
        // exactly unless their exponents span > 29 bits, so the order cannot matter in practice
        double *dst = A.acc_out + (long)(blockIdx.x % A.R_out) * A.Ps;
#pragma unroll
        for (int j = 0; j < C::EPT; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = imap_at(net, Tc, 4 * (tid + j * C::THREADS) + r);
                if (m >= 0) unsafeAtomicAdd(dst + m, (double)part[j][r]);
            }
        if (blockIdx.x == 0)
            for (int e = tid; e < A.zero_len; e += C::THREADS) A.acc_zero[e] = 0.0;
    } else {
        f4 *slab4 = reinterpret_cast<f4 *>(A.slabs + (long)blockIdx.x * C::SLAB);
#pragma unroll
        for (int j = 0; j < C::EPT; ++j) {
            const int e = tid + j * C::THREADS;
            if (e < C::SLAB / 4) slab4[e] = part[j];
        }
    }
#undef WLD
}

// ---------------------------------------------------------------------------
// Cooperative tile kernel, fp32 or fp64 (T).  The TH waves of a GROUP process one 16-sample
// tile together, wave w owning hidden row tile w of layers 1 and 2 (T1 == T2 == TH, T3 == 1).
// Per tile a wave issues 1/TH of the MFMAs, holds only its own weight fragments (registers) and
// its own slice of the gradient accumulators; the NG = WAVES / TH groups of a block are combined
// once at the end.  Exchanges through LDS (double-buffered by tile parity, none when TH == 1):
// y1/Ry1 after layer 0, the layer-2 partial products over the row tiles, and G2.
// fp32 serves the wide policies (2x64: TH = 4); fp64 (v_mfma_f64_16x16x4_f64, every shape) is the
// reference-exact precision mode.  MODE 0: FVP; MODE 1: policy gradient (as fvp_mlp3_kernel);
// MODE 2: CG iteration -- the CG step j-1 -> j (src/TRPO_CG.c:65-103) from the reduced F p_{j-1},
// run redundantly by every block (fixed-order sums: bit-identical in all blocks), p_j staged in
// LDS and gathered into this wave's direction fragments, then FVP j.
// The f64 MFMA's result layout differs from f32's: lane (c, g) register r holds row g + 4r
// (f32: 4g + r), so the fp64 packs use that neuron <-> (g, s) permutation (PT<T>::neu).
// ---------------------------------------------------------------------------
typedef double d4 __attribute__((ext_vector_type(4)));

template <typename T> struct PT;
template <> struct PT<float> {
    typedef f4 V;
    static __device__ __forceinline__ V mfma(float a, float b, V c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    static __host__ __device__ __forceinline__ int neu(int g, int r) { return 4 * g + r; }
    static __device__ __forceinline__ float rsum16(float v) { return rowsum16(v); }
    static __device__ __forceinline__ float th(float x) { return tanh_fast(x); }
    static __device__ __forceinline__ float sg(float x) { return sigmoid_fast(x); }
};
template <> struct PT<double> {
    typedef d4 V;
    static __device__ __forceinline__ V mfma(double a, double b, V c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    static __host__ __device__ __forceinline__ int neu(int g, int r) { return g + 4 * r; }
    static __device__ __forceinline__ double rsum16(double v) { return rowsum16_f64(v); }
    static __device__ __forceinline__ double th(double x) { return tanh64(x); }
    static __device__ __forceinline__ double sg(double x) { return 1.0 / (1.0 + exp(-x)); }
};

__device__ __forceinline__ float fma_t(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ double fma_t(double a, double b, double c) { return __builtin_fma(a, b, c); }
template <typename T, typename V>
__device__ __forceinline__ V actv_fwd(int a, V x, V rx, V &ry) {
    V y;
    if (a == ACT_T) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            y[r] = PT<T>::th(x[r]);
            ry[r] = rx[r] * fma_t(-y[r], y[r], (T)1);   // one rounding, as actv_r
        }
    } else if (a == ACT_S) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            y[r] = PT<T>::sg(x[r]);
            ry[r] = rx[r] * y[r] * ((T)1 - y[r]);
        }
    } else if (a == ACT_O) {
        y = (T)0.1 * x;
        ry = (T)0.1 * rx;
    } else {
        y = x;
        ry = rx;
    }
    return y;
}
// R{y} from R{x} and a cached forward value y (the actv_fwd formulas)
template <typename T, typename V>
__device__ __forceinline__ V actv_r(int a, V y, V rx) {
    V ry;
    if (a == ACT_T) {
#pragma unroll
        for (int r = 0; r < 4; ++r) ry[r] = rx[r] * fma_t(-y[r], y[r], (T)1);
    } else if (a == ACT_S) {
#pragma unroll
        for (int r = 0; r < 4; ++r) ry[r] = rx[r] * y[r] * ((T)1 - y[r]);
    } else if (a == ACT_O) {
        ry = (T)0.1 * rx;
    } else {
        ry = rx;
    }
    return ry;
}
template <typename T, typename V>
__device__ __forceinline__ V actv_bwd(int a, V y, V g) {
    if (a == ACT_T) return g * ((T)1 - y * y);
    if (a == ACT_S) return g * y * ((T)1 - y);
    if (a == ACT_O) return (T)0.1 * g;
    return g;
}
template <typename T>
__device__ __forceinline__ void scr_put_t(T *scr, int row0, typename PT<T>::V t, int c, int g) {
    if constexpr (sizeof(T) == 4) {      // fp32: the scr_put form (one 16-byte store)
        reinterpret_cast<typename PT<T>::V *>(scr)[(row0 >> 4) * 68 + c + 17 * g] = t;
    } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) scr[(row0 + PT<T>::neu(g, r)) * SCR_LD + c] = t[r];
    }
}
template <typename T>
__device__ __forceinline__ typename PT<T>::V scr_get_t(const T *scr, int row0, int c, int g) {
    if constexpr (sizeof(T) == 4) {      // fp32: the scr_get form (transposed reads)
        const T *p = scr + (row0 >> 4) * 272 + 4 * (4 * g + 17 * (c >> 2)) + (c & 3);
        typename PT<T>::V r;
        r[0] = p[0];
        r[1] = p[4];
        r[2] = p[8];
        r[3] = p[12];
        return r;
    } else {
        return *reinterpret_cast<const typename PT<T>::V *>(scr + (row0 + c) * SCR_LD + 4 * g);
    }
}
// a D-layout vector of natural-order values (biases, 1/sigma^2): lane group g, register r -> neu(g, r)
template <typename T>
__device__ __forceinline__ typename PT<T>::V dvec(const T *base, int g) {
    typename PT<T>::V v;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = base[PT<T>::neu(g, r)];
    return v;
}

template <typename T, int T0, int TH>
struct CoopCfg {
    static constexpr bool F64 = sizeof(T) == 8;
    static constexpr int WAVES = F64 ? 4 : 8;   // fp64 TH = 1: one wave per SIMD, room for the forward cache;   // fp64 exchanges: twice the bytes
    static constexpr int GW = TH, NG = WAVES / GW, THREADS = 64 * WAVES;
    // XT (fp32): the y1 and g2 exchange rows padded by one V after every 16 lanes (68 V per 64-lane row),
    // so that RGW1 reads its operands TRANSPOSED straight from them, conflict-free (see the kernel)
    static constexpr bool XT = !F64 && GW > 1;
    static constexpr int XR = XT ? 68 : 64;
    static constexpr int NW = T0 + TH + 4;                 // accumulator vectors per lane per wave
    static constexpr int SLAB = TH * NW * 256;             // T per block partial
    // LDS in V (4 x T) units: exchange buffers [parity][group][row tile][...][lane]
    static constexpr int XB = 0, XB_N = GW > 1 ? 2 * NG * TH * 2 * XR : 0;
    static constexpr int PB = XB + XB_N, PB_N = GW > 1 ? 2 * NG * TH * 2 * 64 : 0;
    static constexpr int GB = PB + PB_N, GB_N = GW > 1 ? 2 * NG * TH * XR : 0;
    static constexpr int EX_V = GB + GB_N;
    static constexpr int SROWS = 16 * (TH + 1 > T0 + 1 ? TH + 1 : T0 + 1);   // per-wave transpose rows
    static constexpr int SCR = SROWS * SCR_LD;             // T per wave
    static constexpr int COMB_V = (NG - 1) * TH * NW * 64; // group-combine dump (aliases exchange)
    static constexpr int MAIN_V = EX_V > COMB_V ? EX_V : COMB_V;
    static constexpr int LDS_BYTES = 4 * (int)sizeof(T) * MAIN_V + (int)sizeof(T) * WAVES * SCR;
    static constexpr int MAIN_BYTES = 4 * (int)sizeof(T) * MAIN_V;   // the fused CG step stages p here
    // parameter-count bound of the shapes this tiling serves (16 T0 -> 16 TH -> 16 TH -> 16)
    static constexpr int PMAX = 256 * (T0 * TH + TH * TH + TH) + 16 * (2 * TH + 2);
    static_assert(TH == 1 || TH == 2 || TH == 4, "TH");
    static_assert(LDS_BYTES <= 160 * 1024, "LDS");
};

// Block-partial (slab) layout of the cooperative kernel.  fp64: the accumulator order in full, NW = T0 + TH + 4
// vectors of 64 lanes per wave.  fp32 (round 5, COMPACT): the RGW0 / RGW1 tiles in full; the RGW2 tile in
// full or, with the narrow output layer (NO, <= 4 outputs), only its 16 lanes of output columns c < 4; the
// three bias rows only from the 4 lanes with c == 0 (after the 16-column sums every other lane holds
// padding) -- 40 % fewer bytes for the FVP epilogue to store and the slab reduce to read (2x64).
template <typename T, int T0, int TH, int NO>
struct CoopSlab {
    static constexpr bool COMPACT = sizeof(T) == 4;
    static constexpr int A2 = NO ? 16 : 64;                           // V of the RGW2 tile
    static constexpr int WV = COMPACT ? (T0 + TH) * 64 + A2 + 12 : (T0 + TH + 4) * 64;   // V per wave
    static constexpr int SLAB = ((TH * WV * 4 + 31) / 32) * 32;      // T per block (reduce: multiple of RS_POS)
};

// slab position -> natural parameter (or -1) for the cooperative kernel's accumulator order
// [wave w][k][lane][r], k over RGW0 tiles (kt0, w), RGW1 tiles (at, w), RGW2 tile (w, 0),
// B1 tile w, B2 tile w, B3 (wave 0 only); p64: the fp64 row permutation.
__device__ __forceinline__ int imap_coop_at(const Net &n, int T0, int TH, int j, bool p64) {
    const int NW = T0 + TH + 4;
    const int w = j / (NW * 256), rem = j % (NW * 256);
    const int k = rem >> 8, lane = (rem >> 2) & 63, r = rem & 3, c = lane & 15, g = lane >> 4;
    const int nr = p64 ? g + 4 * r : 4 * g + r;
    int i, a, b;
    if (k < T0) { i = 0; a = 16 * k + nr; b = 16 * w + c; }
    else if (k < T0 + TH) { i = 1; a = 16 * (k - T0) + nr; b = 16 * w + c; }
    else if (k == T0 + TH) { i = 2; a = 16 * w + nr; b = c; }
    else {
        const int bi = k - (T0 + TH + 1);                 // 0: B1, 1: B2, 2: B3
        if (c != 0 || (bi == 2 && w != 0)) return -1;
        const int nb = bi == 2 ? nr : 16 * w + nr;
        return nb < n.L[bi + 1] ? n.boff[bi] + nb : -1;
    }
    return (a < n.L[i] && b < n.L[i + 1]) ? n.woff[i] + a * n.L[i + 1] + b : -1;
}

// the same for the fp32 compact slab layout (CoopSlab): position j -> (wave, vector, lane, r) of the full
// accumulator order, then imap_coop_at
__device__ __forceinline__ int imap_coop_slab(const Net &n, int T0, int TH, int no, int j, bool p64) {
    if (p64) return imap_coop_at(n, T0, TH, j, p64);
    const int A2 = no ? 16 : 64, WV = (T0 + TH) * 64 + A2 + 12, NW = T0 + TH + 4;
    const int w = j / (4 * WV), rem = j % (4 * WV);
    if (w >= TH) return -1;                               // the block slab's padding
    const int vi = rem >> 2, r = rem & 3;
    int k, lane;
    if (vi < (T0 + TH) * 64) {
        k = vi >> 6;
        lane = vi & 63;
    } else if (vi < (T0 + TH) * 64 + A2) {
        const int li = vi - (T0 + TH) * 64;
        k = T0 + TH;
        lane = no ? (li >> 2) * 16 + (li & 3) : li;        // (g, c < 4)
    } else {
        const int li = vi - (T0 + TH) * 64 - A2;
        k = T0 + TH + 1 + (li >> 2);                      // B1, B2, B3
        lane = (li & 3) * 16;                             // (g, c = 0)
    }
    return imap_coop_at(n, T0, TH, (w * NW + k) * 256 + lane * 4 + r, false);
}

__global__ void build_imap_coop_kernel(Net n, int T0, int TH, int p64, int no, int *imap, int len) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < len) imap[j] = imap_coop_slab(n, T0, TH, no, j, p64 != 0);
}

// direction-pack element e of the cooperative kernel's tile shape, from a natural-order vector
// (pack arithmetic in registers: measured slightly faster than a table lookup round)
template <typename T, int T0, int TH>
__device__ __forceinline__ T coop_vgather(const Net &net, const double *src, int e) {
    constexpr int Tc[4] = {T0, TH, TH, 1};
    const int m = vmap_at(net, Tc, e, sizeof(T) == 8);
    const double v = src[max(m, 0)];                   // unconditional load (no branch, no drain)
    return m >= 0 ? (T)v : (T)0;
}

// NO (fp32 only): the narrow output layer of fvp_mlp3_kernel (<= 4 outputs): each wave's share of the
// output layer's forward / R-forward on v_mfma_f32_4x4x1_16b_f32 (A operands from FA2 / VFA2 lane
// (c & 3) + 16g), summed over its lane groups by two permlane steps and over the group's waves through
// LDS as before; G2 = W2 G3 for the wave's row tile as a VALU fmaf chain; RGW2 and B3 stay on the
// 16x16x4 contraction (G3 back in rows 4g + r).
template <typename T, int T0, int TH, int ACT, int MODE, int NO = 0>
__global__ void __launch_bounds__((CoopCfg<T, T0, TH>::THREADS))
fvp_coop_kernel(IterArgs A, Net net) {
    using Q = CoopCfg<T, T0, TH>;
    using C = FastCfg<T0, TH, TH, 1>;                      // pack offsets (same fragment packs)
    using V = typename PT<T>::V;
    static_assert(NO == 0 || (sizeof(T) == 4 && NO <= 4), "narrow output layer: fp32, <= 4 outputs");
    // MODE 3 / 4: MODE 0 / 2 on the forward-activation cache (fp32; output activation without y):
    // a wave's y1, y2 row tiles come from the cache a MODE 0 launch wrote, the forward MFMAs are skipped
    constexpr bool FV = MODE != 1, UPD = MODE == 2 || MODE == 4, YC = MODE == 3 || MODE == 4;
    constexpr int T1 = TH, T2 = TH;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    T *ldsT = reinterpret_cast<T *>(lds);
    V *LV = reinterpret_cast<V *>(lds);
    // wave index as a wave-uniform (scalar) value: branches on the lane group are then uniform, so a
    // wave runs only its own group's schedule (the rotated one below) with its own barriers
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int c = lane & 15, g = lane >> 4, grp = wave / Q::GW, w = wave % Q::GW;
    T *scr = ldsT + 4 * Q::MAIN_V + wave * Q::SCR;
    const int ntiles = A.ntiles, n = A.n;
    const V *obs4 = reinterpret_cast<const V *>(A.obs4);
    const V *TP = reinterpret_cast<const V *>(A.tpack);
    const V *VP = reinterpret_cast<const V *>(A.vpack);
    const T *TPs = reinterpret_cast<const T *>(A.tpack);
    const T *VPs = reinterpret_cast<const T *>(A.vpack);
    // the first tile's observations are issued with the prologue loads; later tiles are
    // prefetched one step ahead (clamped: every load unconditional)
    const int gstride = gridDim.x * Q::NG;
    // this group's first tile: block-major (blocks 0, 1, .. take NG consecutive tiles) or, with A.gmaj,
    // group-major (every block's group 0 first): at fewer tiles than groups the busy groups then sit
    // one per block, one wave per SIMD, instead of two per block on half the CUs (round 5)
    const int gbase = A.gmaj ? grp * (int)gridDim.x + (int)blockIdx.x : (int)blockIdx.x * Q::NG + grp;
    V xn[T0];
    [[maybe_unused]] V yn1, yn2;                          // cached y1, y2 row tiles of the next tile
    const V *ycl = reinterpret_cast<const V *>(A.yc);
    V *ycs = MODE == 0 ? reinterpret_cast<V *>(A.yc) : nullptr;   // cache writer
    {
        const int tc0 = min(gbase, ntiles - 1);
#pragma unroll
        for (int kt = 0; kt < T0; ++kt) xn[kt] = obs4[(long)(tc0 * 16 + c) * (4 * T0) + kt * 4 + g];
        if constexpr (YC) {
            yn1 = ycl[((long)tc0 * 2 * TH + w) * 64 + lane];
            yn2 = ycl[((long)tc0 * 2 * TH + TH + w) * 64 + lane];
        }
    }
    if (*A.skip) return;                                   // grid-uniform

    const V zero4 = {0, 0, 0, 0};
    // this wave's weight fragments (theta pack), straight to registers
    V fa0[T0], vfa0[T0], fa1[T1], vfa1[T1], fb1[T2];
#pragma unroll
    for (int kt = 0; kt < T0; ++kt) fa0[kt] = TP[C::FA0 / 4 + (w * T0 + kt) * 64 + lane];
#pragma unroll
    for (int kt = 0; kt < T1; ++kt) {
        fa1[kt] = TP[C::FA1 / 4 + (w * T1 + kt) * 64 + lane];
        fb1[kt] = TP[C::FB1 / 4 + (w * T2 + kt) * 64 + lane];
    }
    // narrow output: the output layer's A operands from lane l2 = (c & 3) + 16g, its per-output vectors
    // (bias, 1/sigma^2, ...) for outputs 0..3 in every lane group (g2 = 0)
    const int l2 = NO ? (c & 3) + 16 * g : lane, g2 = NO ? 0 : g;
    const V fa2 = TP[C::FA2 / 4 + w * 64 + l2];
    const V fb2 = NO ? zero4 : TP[C::FB2 / 4 + w * 64 + lane];
    [[maybe_unused]] V w2n[4];                             // NO: W2[16w + 4g + r][0..3] (FB2 lane 4g + r)
    if constexpr (NO) {
#pragma unroll
        for (int r = 0; r < 4; ++r) w2n[r] = TP[C::FB2 / 4 + w * 64 + 4 * g + r];
    }
    const V b0w = dvec<T>(TPs + C::BI0 + 16 * w, g), b1w = dvec<T>(TPs + C::BI1 + 16 * w, g);
    const V b2 = dvec<T>(TPs + C::BI2, g2), iv = dvec<T>(TPs + C::IV, g2);
    V vfa2, vb0w, vb1w, vb2;
    if constexpr (UPD) {
        // ---- CG step j-1 -> j; z = F p_{j-1} arrives reduced (un-normalised) in acc_in ----
        constexpr int EP = (Q::PMAX + Q::THREADS - 1) / Q::THREADS;
        // p_j, then the block-sum and basis-dot scratch, alias the tile exchange buffers (the fused
        // path requires MAIN_BYTES >= 8 (P + 2 + COOP_SH_EXTRA), see trpo_dev_create)
        double *sp = reinterpret_cast<double *>(lds);
        double *shc = sp + ((A.P + 1) & ~1);               // block_sums_dpp<2> | <2>, <= 8 waves
        double *shq = shc + 128;                           // streaming basis dots (reorthogonalisation)
        const CgSt sin = *A.st_in;
        const double cn = A.ctl->n_total, clam = A.ctl->damping, cth = A.ctl->resth;
        const int cmax = A.ctl->maxiter;
        const bool b0 = blockIdx.x == 0;
        double pv[EP], rv[EP], zv[EP], xv[EP];
#pragma unroll
        for (int e = 0; e < EP; ++e) {                     // every load unconditional (clamped)
            const int q = tid + e * Q::THREADS, qc = min(q, A.P - 1), qz = min(q, A.nw - 1);
            const double p0 = A.p_in[qc], r0 = A.r_in[qc], x0 = A.x[b0 ? qc : 0], z0 = A.acc_in[qz];
            const bool in = q < A.P;
            pv[e] = in ? p0 : 0.0;
            rv[e] = in ? r0 : 0.0;
            xv[e] = (in && b0) ? x0 : 0.0;
            zv[e] = q < A.nw ? z0 : 0.0;
        }
        double s1[2] = {0.0, 0.0};
#pragma unroll
        for (int e = 0; e < EP; ++e) {                     // z = sum/N + lambda p; log-std block 2p + lambda p
            const int q = tid + e * Q::THREADS;
            zv[e] = (q < A.nw ? zv[e] / cn : 2.0 * pv[e]) + clam * pv[e];
            s1[0] += pv[e] * zv[e];
            s1[1] += rv[e] * zv[e];
        }
        const bool ro = A.reorth && sin.rdotr > 0.0;
        if (ro && A.nq > 0) qdots_stage1<EP>((const T *)A.q, (const T *)A.qz, A.P, A.Ps, A.nq, zv, Q::THREADS, shq);
        block_sums_dpp<2, Q::THREADS / 64>(s1, shc);
        const double alpha = sin.rdotr / s1[0];
        // residual reorthogonalisation (see QCAP): along r itself, then along the stored basis
        const double cr = ro ? (sqrt(sin.rdotr) - alpha * (s1[1] / sqrt(sin.rdotr))) / sqrt(sin.rdotr) : 0.0;
#pragma unroll
        for (int e = 0; e < EP; ++e) {
            const double r0 = rv[e];
            xv[e] += alpha * pv[e];
            rv[e] -= alpha * zv[e];
            rv[e] -= cr * r0;
        }
        double cs = cr * cr * sin.rdotr;
        if (ro && A.nq > 0)
            cs += qcorrect<EP>((const T *)A.q, (const T *)A.qz, A.P, A.Ps, A.nq, Q::THREADS, shq, alpha, rv);
        double s2[2] = {0.0, 0.0};
#pragma unroll
        for (int e = 0; e < EP; ++e) {
            s2[0] += rv[e] * rv[e];
            s2[1] += xv[e] * xv[e];
        }
        block_sums_dpp<2, Q::THREADS / 64>(s2, shc + 64);
        const double nr = s2[0], beta = nr / sin.rdotr;
#pragma unroll
        for (int e = 0; e < EP; ++e) {
            const int q = tid + e * Q::THREADS;
            if (q < A.P) {
                const double pn = rv[e] + beta * pv[e];
                sp[q] = pn;
                if (b0) {
                    A.p_out[q] = pn;
                    A.r_out[q] = rv[e];
                    A.x[q] = xv[e];
                }
            }
        }
        const int it = sin.iter + 1;
        const int done = (nr < cth || it >= cmax) ? 1 : 0;
        if (b0 && A.reorth) qstore<EP>((T *)A.q, A.P, A.Ps, it, nr, rv, Q::THREADS);
        if (b0 && tid == 0) {
            A.st_out->rdotr = nr;
            A.st_out->xx = s2[1];
            A.st_out->iter = it;
            A.hist[2 * it] = nr;
            A.hist[2 * it + 1] = sqrt(s2[1]);
            A.ctl->rdotr = nr;
            A.ctl->iter = it;
            A.ctl->done = done;
            note_orth(&A.ctl->orth, cs, nr);
            if (it <= CG_AMAX) A.ctl->alpha[it - 1] = alpha;
        }
        if (done) return;                                  // block-uniform
        __syncthreads();
        // this wave's direction fragments gathered from p_j (pack order -> parameter: vmap_at)
        auto vget = [&](int e) -> T { return coop_vgather<T, T0, TH>(net, sp, e); };
#pragma unroll
        for (int kt = 0; kt < T0; ++kt)
#pragma unroll
            for (int s = 0; s < 4; ++s) vfa0[kt][s] = vget(C::VFA0 + ((w * T0 + kt) * 64 + lane) * 4 + s);
#pragma unroll
        for (int kt = 0; kt < T1; ++kt)
#pragma unroll
            for (int s = 0; s < 4; ++s) vfa1[kt][s] = vget(C::VFA1 + ((w * T1 + kt) * 64 + lane) * 4 + s);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            vfa2[s] = vget(C::VFA2 + (w * 64 + l2) * 4 + s);
            vb0w[s] = vget(C::VB0 + 16 * w + PT<T>::neu(g, s));
            vb1w[s] = vget(C::VB1 + 16 * w + PT<T>::neu(g, s));
            vb2[s] = vget(C::VB2 + PT<T>::neu(g2, s));
        }
        __syncthreads();                                   // LDS goes back to the tile exchanges
    } else if (FV && A.v_nat) {                            // plain FVP of a natural-order direction
        auto vget = [&](int e) -> T { return coop_vgather<T, T0, TH>(net, A.v_nat, e); };
#pragma unroll
        for (int kt = 0; kt < T0; ++kt)
#pragma unroll
            for (int s = 0; s < 4; ++s) vfa0[kt][s] = vget(C::VFA0 + ((w * T0 + kt) * 64 + lane) * 4 + s);
#pragma unroll
        for (int kt = 0; kt < T1; ++kt)
#pragma unroll
            for (int s = 0; s < 4; ++s) vfa1[kt][s] = vget(C::VFA1 + ((w * T1 + kt) * 64 + lane) * 4 + s);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            vfa2[s] = vget(C::VFA2 + (w * 64 + l2) * 4 + s);
            vb0w[s] = vget(C::VB0 + 16 * w + PT<T>::neu(g, s));
            vb1w[s] = vget(C::VB1 + 16 * w + PT<T>::neu(g, s));
            vb2[s] = vget(C::VB2 + PT<T>::neu(g2, s));
        }
        if (A.init && blockIdx.x == gridDim.x - 1) {
            // the CG start of the distributed path fused into its first FVP (v_nat = b): the block
            // with the fewest tiles writes x = 0, r = p = b, |b|^2, q_0 = b / |b| and the control state
            // (cg_init_kernel's work, src/TRPO_CG.c:19-43), so the solve needs no init launch
            #pragma clang fp contract(off)
            constexpr int EP = (Q::PMAX + Q::THREADS - 1) / Q::THREADS;
            double bv[EP], red[1] = {0.0};
#pragma unroll
            for (int e = 0; e < EP; ++e) {
                const int q = tid + e * Q::THREADS;
                const double b0 = A.b_init[min(q, A.P - 1)];
                bv[e] = q < A.P ? b0 : 0.0;
                red[0] += bv[e] * bv[e];
            }
            block_sums_dpp<1, Q::THREADS / 64>(red, reinterpret_cast<double *>(lds));
            const double rr = red[0];
#pragma unroll
            for (int e = 0; e < EP; ++e) {
                const int q = tid + e * Q::THREADS;
                if (q < A.P) {
                    A.p_out[q] = bv[e];
                    A.r_out[q] = bv[e];
                    A.x[q] = 0.0;
                }
            }
            if (A.reorth) qstore<EP>((T *)A.q, A.P, A.Ps, 0, rr, bv, Q::THREADS);     // q_0 = b / |b|
            if (tid == 0) {
                A.st_out->rdotr = rr;
                A.st_out->xx = 0.0;
                A.st_out->iter = 0;
                A.hist[0] = rr;
                A.hist[1] = 0.0;
                A.ctl->maxiter = A.init_maxiter;
                A.ctl->resth = A.init_resth;
                A.ctl->rdotr = rr;
                A.ctl->iter = 0;
                A.ctl->orth = 0.0;
                A.ctl->done = (rr < A.init_resth || A.init_maxiter == 0) ? 1 : 0;
            }
            __syncthreads();                               // the LDS scratch goes back to the tiles
        }
    } else {
#pragma unroll
        for (int kt = 0; kt < T0; ++kt) vfa0[kt] = FV ? VP[C::VFA0 / 4 + (w * T0 + kt) * 64 + lane] : zero4;
#pragma unroll
        for (int kt = 0; kt < T1; ++kt) vfa1[kt] = FV ? VP[C::VFA1 / 4 + (w * T1 + kt) * 64 + lane] : zero4;
        vfa2 = FV ? VP[C::VFA2 / 4 + w * 64 + l2] : zero4;
        vb0w = FV ? dvec<T>(VPs + C::VB0 + 16 * w, g) : zero4;
        vb1w = FV ? dvec<T>(VPs + C::VB1 + 16 * w, g) : zero4;
        vb2 = FV ? dvec<T>(VPs + C::VB2, g2) : zero4;
    }

    const int a1 = ACT >= 0 ? (ACT & 3) : net.act[1];
    const int a2 = ACT >= 0 ? ((ACT >> 2) & 3) : net.act[2];
    const int a3 = ACT >= 0 ? ((ACT >> 4) & 3) : net.act[3];
    const bool y3_needed = act_needs_y(a3);

    V accW0[T0], accW1[T1], accW2 = zero4, sB1 = zero4, sB2 = zero4, sB3 = zero4;
#pragma unroll
    for (int k = 0; k < T0; ++k) accW0[k] = zero4;
#pragma unroll
    for (int k = 0; k < T1; ++k) accW1[k] = zero4;

    // every wave of the block runs the same number of tile steps (barriers inside)
    const int nsteps = (ntiles + gstride - 1) / gstride;
    // One tile step is four segments separated by the group's three LDS exchanges (block barriers):
    //   S0 layer 0 (R chain) -> [y1/r1 rows] -> S1 layer 1, the layer-2 partial over this row tile ->
    //   [layer-2 partials] -> S2 G3, RGW2, G2 -> [g2 rows] -> S3 G1, RGW1, RGW0.
    // (Round 5 measured running the second lane group one barrier later, so that the two waves of a
    // SIMD would pair a heavy segment with a light one: slower -- 451 vs 444 us per 2x64 solve at 50k --
    // and it is not kept; profiles/HISTORY.md.)
    [[maybe_unused]] V x0[T0], yc1, yc2, y1w, r1w, y1[T1], r1[T1], y2w, r2w, a3p, r3p, r3q, g2w;
    // NOV (round 5, fp32 narrow output): RGW2 as per-lane VALU partials over the lane's own sample column
    // (hidden 16w + 4g + r x output o), summed over the 16 columns once in the epilogue -- 16 FMAs per tile
    // instead of two LDS transposes and 4 MFMAs whose 16 columns carried <= 4 outputs
    constexpr bool NOV = NO != 0 && sizeof(T) == 4;
    [[maybe_unused]] float acc2v[4][NO > 0 ? NO : 1];
    if constexpr (NOV) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int o = 0; o < (NO > 0 ? NO : 1); ++o) acc2v[r][o] = 0.0f;
    }
    auto seg0 = [&](int step) __attribute__((always_inline)) {
        const int tile = step * gstride + gbase;
        const int par = step & 1;
        V *xb = LV + Q::XB + ((par * Q::NG + grp) * TH) * 2 * Q::XR;   // [row tile][2][64 (+4 pad)]
        const int xl = Q::XT ? lane + (lane >> 4) : lane;               // this lane's V in such a row
#pragma unroll
        for (int kt = 0; kt < T0; ++kt) x0[kt] = xn[kt];
        if constexpr (YC) {
            yc1 = yn1;
            yc2 = yn2;
        }
        {
            const int tn = min(tile + gstride, ntiles - 1);
#pragma unroll
            for (int kt = 0; kt < T0; ++kt) xn[kt] = obs4[(long)(tn * 16 + c) * (4 * T0) + kt * 4 + g];
            if constexpr (YC) {
                yn1 = ycl[((long)tn * 2 * TH + w) * 64 + lane];
                yn2 = ycl[((long)tn * 2 * TH + TH + w) * 64 + lane];
            }
            __builtin_amdgcn_sched_barrier(0);             // keep the prefetch here (see fvp_mlp3_kernel)
        }
        // ---- layer 0, row tile w ----
        V a = b0w, ra = vb0w;
#pragma unroll
        for (int kt = 0; kt < T0; ++kt)
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                if constexpr (!YC) a = PT<T>::mfma(fa0[kt][s], x0[kt][s], a);
                if constexpr (FV) ra = PT<T>::mfma(vfa0[kt][s], x0[kt][s], ra);
            }
        if constexpr (YC) {
            y1w = yc1;
            r1w = actv_r<T>(a1, y1w, ra);
        } else {
            y1w = actv_fwd<T>(a1, a, ra, r1w);
            if (ycs && tile < ntiles) ycs[((long)tile * 2 * TH + w) * 64 + lane] = y1w;
        }
        if constexpr (Q::GW > 1) {
            xb[w * 2 * Q::XR + xl] = y1w;
            if constexpr (FV) xb[w * 2 * Q::XR + Q::XR + xl] = r1w;
        }
    };
    auto seg1 = [&](int step) __attribute__((always_inline)) {
        const int tile = step * gstride + gbase;
        const int par = step & 1;
        V *xb = LV + Q::XB + ((par * Q::NG + grp) * TH) * 2 * Q::XR;
        V *pb = LV + Q::PB + ((par * Q::NG + grp) * TH) * 128;
        const int xl = Q::XT ? lane + (lane >> 4) : lane;
        if constexpr (Q::GW > 1) {
#pragma unroll
            for (int kt = 0; kt < T1; ++kt) {
                y1[kt] = xb[kt * 2 * Q::XR + xl];
                r1[kt] = FV ? xb[kt * 2 * Q::XR + Q::XR + xl] : zero4;
            }
        } else {
            y1[0] = y1w;
            r1[0] = r1w;
        }
        // ---- layer 1, row tile w ----
        V a = b1w, ra = vb1w, rb = zero4;
#pragma unroll
        for (int kt = 0; kt < T1; ++kt)
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                if constexpr (!YC) a = PT<T>::mfma(fa1[kt][s], y1[kt][s], a);
                if constexpr (FV) {
                    ra = PT<T>::mfma(fa1[kt][s], r1[kt][s], ra);
                    rb = PT<T>::mfma(vfa1[kt][s], y1[kt][s], rb);
                }
            }
        if constexpr (YC) {
            y2w = yc2;
            r2w = actv_r<T>(a2, y2w, ra + rb);
        } else {
            y2w = actv_fwd<T>(a2, a, ra + rb, r2w);
            if (ycs && tile < ntiles) ycs[((long)tile * 2 * TH + TH + w) * 64 + lane] = y2w;
        }
        // ---- layer 2: this wave's share (input row tile w), summed over the group in S2 ----
        a3p = zero4;
        r3p = zero4;
        r3q = zero4;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            if constexpr (NO) {
                if (!YC && y3_needed) a3p = MFMA4(fa2[s], y2w[s], a3p);
                if constexpr (FV) {
                    r3p = MFMA4(fa2[s], r2w[s], r3p);
                    r3q = MFMA4(vfa2[s], y2w[s], r3q);
                }
            } else {
                if (!YC && y3_needed) a3p = PT<T>::mfma(fa2[s], y2w[s], a3p);   // YC: y3 never needed
                if constexpr (FV) {
                    r3p = PT<T>::mfma(fa2[s], r2w[s], r3p);
                    r3q = PT<T>::mfma(vfa2[s], y2w[s], r3q);
                }
            }
        }
        if constexpr (NO) {                                // the wave's 16 hidden neurons: sum the lane groups
            if (!YC && y3_needed) a3p = rowgroup_sum4(a3p);
            r3p = FV ? rowgroup_sum4(r3p + r3q) : zero4;
            r3q = zero4;
        }
        if constexpr (Q::GW > 1) {
            pb[w * 128 + lane] = a3p;
            pb[w * 128 + 64 + lane] = r3p + r3q;
        }
    };
    auto seg2 = [&](int step) __attribute__((always_inline)) {
        const int tile = step * gstride + gbase;
        const int tc = min(tile, ntiles - 1);
        const bool live = tile < ntiles && tc * 16 + c < n;
        const int par = step & 1;
        V *pb = LV + Q::PB + ((par * Q::NG + grp) * TH) * 128;
        V *gb = LV + Q::GB + ((par * Q::NG + grp) * TH) * Q::XR;        // [row tile][64 (+4 pad)]
        const int xl = Q::XT ? lane + (lane >> 4) : lane;
        V x3 = b2, rx3 = vb2;
        if constexpr (Q::GW > 1) {
#pragma unroll
            for (int kt = 0; kt < TH; ++kt) {              // fixed order
                x3 += pb[kt * 128 + lane];
                rx3 += pb[kt * 128 + 64 + lane];
            }
        } else {
            x3 += a3p;
            rx3 += r3p + r3q;
        }
        V r3, g3;
        const V y3 = actv_fwd<T>(a3, x3, rx3, r3);
        if constexpr (FV) {
            g3 = actv_bwd<T>(a3, y3, r3 * iv);
        } else {
            const V dm = dvec<T>(reinterpret_cast<const T *>(A.pg_d4) + (long)(tc * 16 + c) * 16, g2);
            const T adv = reinterpret_cast<const T *>(A.pg_adv)[tc * 16 + c];
            g3 = actv_bwd<T>(a3, y3, (adv * dm) * dvec<T>(reinterpret_cast<const T *>(A.pg_iv4), g2));
        }
        g3 = live ? g3 : zero4;
        // NO: every lane group holds outputs 0..3; the contractions below want rows 4g + r
        const V g3m = (NO && g != 0) ? zero4 : g3;
        if (w == 0) sB3 += g3m;
        // ---- RGW2 tile (w, 0) += Y2_w . G3^T ----
        if constexpr (NOV) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int o = 0; o < (NO > 0 ? NO : 1); ++o) acc2v[r][o] = fmaf((float)y2w[r], (float)g3[o], acc2v[r][o]);
        } else {
            scr_put_t<T>(scr, 0, y2w, c, g);
            scr_put_t<T>(scr, 16, g3m, c, g);
            const V ya = scr_get_t<T>(scr, 0, c, g), gg = scr_get_t<T>(scr, 16, c, g);
#pragma unroll
            for (int s = 0; s < 4; ++s) accW2 = PT<T>::mfma(ya[s], gg[s], accW2);
        }
        // ---- G2 row tile w = act2'(W2 G3) ----
        V t = zero4;
        if constexpr (NO) {
            // the fmaf chain over the outputs a 16x16x4 MFMA forms (its padded rows added zeros)
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int o = 0; o < NO; ++o) t[r] = fmaf(w2n[r][o], g3[o], t[r]);
        } else {
#pragma unroll
            for (int s = 0; s < 4; ++s) t = PT<T>::mfma(fb2[s], g3[s], t);
        }
        g2w = actv_bwd<T>(a2, y2w, t);
        sB2 += g2w;
        if constexpr (Q::GW > 1) gb[w * Q::XR + xl] = g2w;
    };
    auto seg3 = [&](int step) __attribute__((always_inline)) {
        const int par = step & 1;
        V *xb = LV + Q::XB + ((par * Q::NG + grp) * TH) * 2 * Q::XR;
        V *gb = LV + Q::GB + ((par * Q::NG + grp) * TH) * Q::XR;
        const int xl = Q::XT ? lane + (lane >> 4) : lane;
        V g2[T2];
        if constexpr (Q::GW > 1) {
#pragma unroll
            for (int kt = 0; kt < T2; ++kt) g2[kt] = gb[kt * Q::XR + xl];
        } else {
            g2[0] = g2w;
        }
        // ---- G1 row tile w = act1'(W1 G2) ----
        V t = zero4;
#pragma unroll
        for (int kt = 0; kt < T2; ++kt)
#pragma unroll
            for (int s = 0; s < 4; ++s) t = PT<T>::mfma(fb1[kt][s], g2[kt][s], t);
        const V g1w = actv_bwd<T>(a1, y1w, t);
        sB1 += g1w;
        // ---- RGW1 tiles (at, w) += Y1_at . G2_w^T ----
        if constexpr (Q::XT) {
            // both operands read transposed from the exchange rows, which hold them in the D layout
            // (lane l = sample + 16 (feature / 4), register feature % 4; +1 V per 16 lanes): lane (c, g)
            // needs feature c of samples 4g .. 4g + 3, i.e. floats 4 (4g + s + 17 (c / 4)) + c % 4 of the
            // row -- stride 4 floats in s (ds_read2_b32 pairs), banks 16g + 4 (c / 4) + c % 4 + 4s mod 64:
            // all 64 lanes distinct.  Same products in the same order as the scratch transpose below.
            const T *xbf = reinterpret_cast<const T *>(xb), *gbf = reinterpret_cast<const T *>(gb);
            const int bt = 4 * (4 * g + 17 * (c >> 2)) + (c & 3);
            V gg;
#pragma unroll
            for (int s = 0; s < 4; ++s) gg[s] = gbf[w * 4 * Q::XR + bt + 4 * s];
#pragma unroll
            for (int at = 0; at < T1; ++at) {
                V ya;
#pragma unroll
                for (int s = 0; s < 4; ++s) ya[s] = xbf[at * 8 * Q::XR + bt + 4 * s];
#pragma unroll
                for (int s = 0; s < 4; ++s) accW1[at] = PT<T>::mfma(ya[s], gg[s], accW1[at]);
            }
        } else {
#pragma unroll
            for (int at = 0; at < T1; ++at) scr_put_t<T>(scr, 16 * at, y1[at], c, g);
            scr_put_t<T>(scr, 16 * T1, g2w, c, g);
            {
                const V gg = scr_get_t<T>(scr, 16 * T1, c, g);
#pragma unroll
                for (int at = 0; at < T1; ++at) {
                    const V ya = scr_get_t<T>(scr, 16 * at, c, g);
#pragma unroll
                    for (int s = 0; s < 4; ++s) accW1[at] = PT<T>::mfma(ya[s], gg[s], accW1[at]);
                }
            }
        }
        // ---- RGW0 tiles (kt0, w) += X0_kt0 . G1_w^T ----
#pragma unroll
        for (int kt = 0; kt < T0; ++kt) scr_put_t<T>(scr, 16 * kt, x0[kt], c, g);
        scr_put_t<T>(scr, 16 * T0, g1w, c, g);
        {
            const V gg = scr_get_t<T>(scr, 16 * T0, c, g);
#pragma unroll
            for (int kt = 0; kt < T0; ++kt) {
                const V ya = scr_get_t<T>(scr, 16 * kt, c, g);
#pragma unroll
                for (int s = 0; s < 4; ++s) accW0[kt] = PT<T>::mfma(ya[s], gg[s], accW0[kt]);
            }
        }
    };
    // the group exchanges' barrier (none with one wave per group)
    auto xsync = [&]() __attribute__((always_inline)) {
        if constexpr (Q::GW > 1) __syncthreads();
    };
    for (int step = 0; step < nsteps; ++step) {
        // a group past the last tile skips its segments (wave-uniform; it still joins the block's
        // barriers): its masked products would add exact zeros, so only its SIMD partner's time changes
        const bool act = step * gstride + gbase < ntiles;
        if (act) seg0(step);
        xsync();
        if (act) seg1(step);
        xsync();
        if (act) seg2(step);
        xsync();
        if (act) seg3(step);
    }

    // ---- epilogue: bias sums over the sample columns, NG-way group combine, block partial ----
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        sB1[r] = PT<T>::rsum16(sB1[r]);
        sB2[r] = PT<T>::rsum16(sB2[r]);
        sB3[r] = PT<T>::rsum16(sB3[r]);
    }
    if constexpr (NOV) {
        // the 16 sample columns of each RGW2 partial summed (every lane of the row gets the total); lane
        // (c, g) keeps output o = c in register r, the accumulator layout of the MFMA form
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float v = 0.0f;
#pragma unroll
            for (int o = 0; o < (NO > 0 ? NO : 1); ++o) {
                const float t = rowsum16(acc2v[r][o]);
                v = c == o ? t : v;
            }
            accW2[r] = v;
        }
    }
    V acc[Q::NW];
    {
        int k = 0;
#pragma unroll
        for (int i = 0; i < T0; ++i) acc[k++] = accW0[i];
#pragma unroll
        for (int i = 0; i < T1; ++i) acc[k++] = accW1[i];
        acc[k++] = accW2;
        acc[k++] = sB1;
        acc[k++] = sB2;
        acc[k++] = sB3;
    }
    if constexpr (Q::NG > 1) {
        __syncthreads();                                   // exchange buffers are free now
        if (grp > 0) {
#pragma unroll
            for (int k = 0; k < Q::NW; ++k) LV[(((grp - 1) * TH + w) * Q::NW + k) * 64 + lane] = acc[k];
        }
        __syncthreads();
    }
    if (grp == 0) {
#pragma unroll
        for (int q = 1; q < Q::NG; ++q)
#pragma unroll
            for (int k = 0; k < Q::NW; ++k) acc[k] += LV[(((q - 1) * TH + w) * Q::NW + k) * 64 + lane];
        if (A.acc_out) {
            double *dst = A.acc_out + (long)(blockIdx.x % A.R_out) * A.Ps;
#pragma unroll
            for (int k = 0; k < Q::NW; ++k)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int m = imap_coop_at(net, T0, TH, (w * Q::NW + k) * 256 + lane * 4 + r, Q::F64);
                    if (m >= 0) unsafeAtomicAdd(dst + m, (double)acc[k][r]);
                }
        } else {
            using SL = CoopSlab<T, T0, TH, NO>;
            V *slab4 = reinterpret_cast<V *>(reinterpret_cast<T *>(A.slabs) + (long)blockIdx.x * SL::SLAB);
            if constexpr (SL::COMPACT) {
                V *base = slab4 + w * SL::WV;
#pragma unroll
                for (int k = 0; k < T0 + TH; ++k) base[k * 64 + lane] = acc[k];
                if constexpr (NO != 0) {
                    if (c < 4) base[(T0 + TH) * 64 + g * 4 + c] = acc[T0 + TH];
                } else {
                    base[(T0 + TH) * 64 + lane] = acc[T0 + TH];
                }
                if (c == 0) {
#pragma unroll
                    for (int i = 0; i < 3; ++i) base[(T0 + TH) * 64 + SL::A2 + i * 4 + g] = acc[T0 + TH + 1 + i];
                }
            } else {
#pragma unroll
                for (int k = 0; k < Q::NW; ++k) slab4[(w * Q::NW + k) * 64 + lane] = acc[k];
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Generic FVP kernel: any depth, any widths (one thread per sample; T = float, or double in the fp64
// precision mode, which runs the reference's own arithmetic: fp64 products, tanh64).
// Per-sample activations live in a block-private global scratch laid out
// [row][256] so that every access is coalesced across the block.
// ---------------------------------------------------------------------------
constexpr int GEN_T = 256;

template <typename T>
__global__ void __launch_bounds__(GEN_T)
fvp_generic_kernel(const T *__restrict__ obs, int n, const T *__restrict__ th, const T *__restrict__ v,
                   const T *__restrict__ iv, T *__restrict__ scratch, int srows, T *__restrict__ slabs,
                   int sstride, Net net, const int *__restrict__ skip) {
    if (*skip) return;
    const int tid = threadIdx.x;
    T *Y = scratch + (long)blockIdx.x * 3 * srows * GEN_T;
    T *RY = Y + (long)srows * GEN_T;
    T *RG = RY + (long)srows * GEN_T;
    int roff[MAXL + 1];
    roff[0] = 0;
    for (int i = 0; i < net.nl; ++i) roff[i + 1] = roff[i] + net.L[i];
    T *slab = slabs + (long)blockIdx.x * sstride;
    const int nw = net.P - net.A;
    for (int q = tid; q < nw; q += GEN_T) slab[q] = T(0);

    const int npass = (n + GEN_T - 1) / GEN_T;
    for (int pass = blockIdx.x; pass < npass; pass += gridDim.x) {
        const int s = pass * GEN_T + tid;
        const bool live = s < n;
        for (int k = 0; k < net.L[0]; ++k) {
            Y[k * GEN_T + tid] = live ? obs[(long)s * net.L[0] + k] : T(0);
            RY[k * GEN_T + tid] = T(0);
        }
        for (int i = 0; i + 1 < net.nl; ++i) {
            const int in = net.L[i], out = net.L[i + 1];
            const T *W = th + net.woff[i], *B = th + net.boff[i];
            const T *VWp = v + net.woff[i], *VB = v + net.boff[i];
            for (int j = 0; j < out; ++j) {
                T x = B[j], rx = VB[j];
                for (int k = 0; k < in; ++k) {
                    const T yk = Y[(roff[i] + k) * GEN_T + tid], ryk = RY[(roff[i] + k) * GEN_T + tid];
                    x += yk * W[k * out + j];
                    rx += ryk * W[k * out + j];
                    rx += yk * VWp[k * out + j];
                }
                const T y = act_y(net.act[i + 1], x);
                Y[(roff[i + 1] + j) * GEN_T + tid] = y;
                RY[(roff[i + 1] + j) * GEN_T + tid] = act_r(net.act[i + 1], y, rx);
            }
        }
        const int last = net.nl - 1;
        for (int j = 0; j < net.A; ++j) {
            const T y = Y[(roff[last] + j) * GEN_T + tid];
            const T gg = act_r(net.act[last], y, RY[(roff[last] + j) * GEN_T + tid] * iv[j]);
            RG[(roff[last] + j) * GEN_T + tid] = live ? gg : T(0);
        }
        for (int i = last; i >= 2; --i) {
            const int cur = net.L[i], prev = net.L[i - 1];
            const T *W = th + net.woff[i - 1];
            for (int j = 0; j < prev; ++j) {
                T t = T(0);
                for (int k = 0; k < cur; ++k) t += W[j * cur + k] * RG[(roff[i] + k) * GEN_T + tid];
                RG[(roff[i - 1] + j) * GEN_T + tid] = act_r(net.act[i - 1], Y[(roff[i - 1] + j) * GEN_T + tid], t);
            }
        }
        __syncthreads();
        // contraction over the 256 samples of this pass, one parameter per thread
        for (int q = tid; q < nw; q += GEN_T) {
            int i = 0;
            while (i + 2 < net.nl && q >= net.woff[i + 1]) ++i;
            const int in = net.L[i], out = net.L[i + 1];
            const int local = q - net.woff[i];
            T acc = T(0);
            if (local < in * out) {
                const int a = local / out, b = local % out;
                const T *ya = Y + (long)(roff[i] + a) * GEN_T, *gb = RG + (long)(roff[i + 1] + b) * GEN_T;
                for (int t = 0; t < GEN_T; ++t) acc += ya[t] * gb[t];
            } else {
                const T *gb = RG + (long)(roff[i + 1] + local - in * out) * GEN_T;
                for (int t = 0; t < GEN_T; ++t) acc += gb[t];
            }
            slab[q] += acc;
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Cross-block reduction (fp64, fixed order) -> zacc[P-A]
// block = 64 parameters x 16 slab groups
// ---------------------------------------------------------------------------
// zacc[imap[j]] = sum over blocks of slabs[b][j], fp64, fixed order; j runs over the slab
// layout (contiguous).  A block of 256 threads owns RS_POS consecutive slab positions; each
// thread loads 16 B (4 fp32 / 2 fp64 positions) from every SG-th block partial (all its loads in
// flight together), then the SG sub-sums are added in a fixed order through LDS.
constexpr int RS_POS = 32, RS_THREADS = 256;
template <typename ST>
__global__ void __launch_bounds__(RS_THREADS)
reduce_slabs_kernel(const ST *__restrict__ slabs, int G, int slab, const int *__restrict__ imap,
                    double *__restrict__ zacc, const int *__restrict__ skip, const double *__restrict__ vin,
                    double *__restrict__ zout, const Ctl *__restrict__ ctl, int nw, int P,
                    double *__restrict__ zh) {
    constexpr int VE = 16 / sizeof(ST), LP = RS_POS / VE, SG = RS_THREADS / LP, NLD = 256 / SG;
    typedef ST VT __attribute__((ext_vector_type(VE)));
    __shared__ double part[SG][RS_POS + 1];
    const int t = threadIdx.x, lp = t % LP, sg = t / LP;
    const int j0 = blockIdx.x * RS_POS + lp * VE;        // slab % RS_POS == 0 (multiple of 256)
    const int m = t < RS_POS ? imap[blockIdx.x * RS_POS + t] : -1;
    if (*skip) return;
    double s[VE];
#pragma unroll
    for (int e = 0; e < VE; ++e) s[e] = 0.0;
    // the FVP epilogue's direction value vin[m] is gathered between the first slab loads and their sums (one
    // round trip, not two); slab loads clamped and masked by a multiply (+-0 adds nothing), so the compiler
    // can count them instead of draining exec-masked loads (round 5, as reduce_dots_kernel)
    // (the first round runs in every thread, also where sg >= G, so that every thread gathers its vin[m])
    double vm = 0.0;
    for (int b0 = sg, r0 = 1; r0 || b0 < G; b0 += SG * NLD, r0 = 0) {
        VT v[NLD];
#pragma unroll
        for (int k = 0; k < NLD; ++k) {
            const int b = b0 + SG * k;
            v[k] = *reinterpret_cast<const VT *>(slabs + (long)min(b, G - 1) * slab + j0) * (ST)(b < G ? 1 : 0);
        }
        if (r0 && zout) vm = vin[max(m, 0)];
#pragma unroll
        for (int k = 0; k < NLD; ++k)
#pragma unroll
            for (int e = 0; e < VE; ++e) s[e] += (double)v[k][e];
    }
#pragma unroll
    for (int e = 0; e < VE; ++e) part[sg][lp * VE + e] = s[e];
    __syncthreads();
    if (t < RS_POS && m >= 0) {
        double a = 0.0;
#pragma unroll 8
        for (int k = 0; k < SG; ++k) a += part[k][t];
        if (zout) {                                    // fused FVP epilogue
            const double z = a / ctl->n_total + ctl->damping * vm;
            zout[m] = z;
            if (zh) zh[m] = z;                         // also into the caller's mapped host buffer
        } else {
            zacc[m] = a;
        }
    }
    if (zout && blockIdx.x == 0 && t < P - nw) {      // log-std block: 2 v + damping v
        const double vq = vin[nw + t];
        const double z = 2.0 * vq + ctl->damping * vq;
        zout[nw + t] = z;
        if (zh) zh[nw + t] = z;
    }
}

// z = zacc / N + damping * v ; log-std block = 2 v + damping v   (src/TRPO_FVP.c:919-931)
__global__ void fvp_epilogue_kernel(const double *__restrict__ zacc, const double *__restrict__ v,
                                    double *__restrict__ z, int P, int nw, const Ctl *__restrict__ ctl) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= P) return;
    const double vq = v[q];
    z[q] = (q < nw ? zacc[q] / ctl->n_total : 2.0 * vq) + ctl->damping * vq;
}

// the same epilogue from R atomic replicas of the un-normalised sum (fixed replica order)
// The replica set is left zeroed (each element by the thread that consumed it), so standalone FVPs
// need no separate zeroing and the same launch sequence can be replayed from a graph.
// zh (optional): a second copy of z into pinned, device-mapped host memory (the host-level FVP call
// then needs no separate download copy)
__global__ void acc_epilogue_kernel(double *__restrict__ acc, int R, const double *__restrict__ v,
                                    double *__restrict__ z, int P, int Ps, int nw, const Ctl *__restrict__ ctl,
                                    double *__restrict__ zh) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= P) return;
    double a[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) a[r] = acc[(long)min(r, R - 1) * Ps + min(q, nw - 1)];
    double s = a[0];
#pragma unroll
    for (int r = 1; r < 8; ++r) s += r < R ? a[r] : 0.0;
    const double vq = v[q];
    const double zq = (q < nw ? s / ctl->n_total : 2.0 * vq) + ctl->damping * vq;
    z[q] = zq;
    if (zh) zh[q] = zq;
    if (q < nw)
        for (int r = 0; r < R; ++r) acc[(long)r * Ps + q] = 0.0;
}

// ---------------------------------------------------------------------------
// CG (src/TRPO_CG.c:11-113), one 1024-thread block, all fp64, fixed-order sums
// ---------------------------------------------------------------------------

// p -> fragment-order pack (fp32, or fp64 in the fp64 mode) for the next FVP (fast path only;
// vlen == 0 otherwise).  The map entries are loaded up front with the kernel's other loads.
constexpr int VPACK_PER_THREAD = 8;                 // vlen <= 8 * 1024 (checked at context creation)
__device__ __forceinline__ void load_vmap(const int *__restrict__ vmap, int vlen, int (&vm)[VPACK_PER_THREAD]) {
    // unconditional (clamped) loads: a guarded load would drain vmcnt before the next one
#pragma unroll
    for (int k = 0; k < VPACK_PER_THREAD; ++k) {
        const int e = threadIdx.x + k * 1024;
        const int m = vmap[min(e, max(vlen - 1, 0))];
        vm[k] = e < vlen ? m : -1;
    }
}
__device__ __forceinline__ void write_vpack(const double *sp, const int (&vm)[VPACK_PER_THREAD], void *vpack, int vlen,
                                            int f64) {
#pragma unroll
    for (int k = 0; k < VPACK_PER_THREAD; ++k) {
        const int e = threadIdx.x + k * 1024;
        if (e < vlen) {
            const double v = vm[k] >= 0 ? sp[vm[k]] : 0.0;
            if (f64) reinterpret_cast<double *>(vpack)[e] = v;
            else reinterpret_cast<float *>(vpack)[e] = (float)v;
        }
    }
}

// x = 0, r = p = b, state 0; packs p for the first FVP; zeroes the first atomic target.
template <int E, typename QT>
__global__ void __launch_bounds__(1024)
cg_init_kernel(const double *__restrict__ b, double *x, double *r, double *p, int P, Ctl *ctl, CgSt *st,
               double *hist, int maxiter, double resth, const int *__restrict__ vmap, void *vpack,
               int vlen, int f64, double *acc_zero, int zero_len, void *qbuf_v, int Ps) {
    QT *qbuf = reinterpret_cast<QT *>(qbuf_v);
    __shared__ double sh[16];
    extern __shared__ double sp[];
    double bv[E];
    int vm[VPACK_PER_THREAD];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int q = threadIdx.x + e * 1024;
        const double b0 = b[min(q, P - 1)];
        bv[e] = q < P ? b0 : 0.0;
    }
    if (vlen) load_vmap(vmap, vlen, vm);
    for (int e = threadIdx.x; e < zero_len; e += 1024) acc_zero[e] = 0.0;
    double s = 0.0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int q = threadIdx.x + e * 1024;
        if (q < P) {
            x[q] = 0.0;
            r[q] = bv[e];
            p[q] = bv[e];
            if (vlen) sp[q] = bv[e];
            s += bv[e] * bv[e];
        }
    }
    const double rr = block_sum(s, sh);
    qstore<E>(qbuf, P, Ps, 0, rr, bv, 1024);              // q_0 = b / |b| (reorthogonalisation basis; NULL: off)
    if (threadIdx.x == 0) {
        ctl->maxiter = maxiter;
        ctl->resth = resth;
        ctl->rdotr = rr;
        ctl->iter = 0;
        ctl->orth = 0.0;
        st->rdotr = rr;
        st->xx = 0.0;
        st->iter = 0;
        hist[0] = rr;
        hist[1] = 0.0;
        ctl->done = (rr < resth || maxiter == 0) ? 1 : 0;
    }
    write_vpack(sp, vm, vpack, vlen, f64);    // block_sum's barriers ordered the sp writes
}

// One CG step after z = F p is available as R_in fp64 partial-sum replicas (src/TRPO_CG.c:65-103):
// used after the last FVP of a solve, and for every step of the generic (non-fused) path.
// All global loads are issued before the first reduction.
template <int E, typename QT>
__global__ void __launch_bounds__(1024)
cg_update_kernel(const double *__restrict__ acc, int R_in, const double *__restrict__ p_in,
                 const double *__restrict__ r_in, double *p_out, double *r_out, double *x, int P, int nw, Ctl *ctl,
                 const CgSt *st_in, CgSt *st_out, double *hist,
                 const int *__restrict__ vmap, void *vpack, int vlen, int f64,
                 void *qbuf_v, const void *qz_v, int nq, int Ps,
                 double *acc_zero = nullptr, int zero_len = 0) {
    // acc_zero: the atomic target of the NEXT solve's first FVP (which also runs the CG start),
    // zeroed here once this step has consumed its input
    // few elements per thread (small P): the reorthogonalisation basis joins the single load round and
    // the first block reduction (QREG); otherwise the streaming form
    QT *qbuf = reinterpret_cast<QT *>(qbuf_v);
    const QT *qz = reinterpret_cast<const QT *>(qz_v);
    constexpr bool QREG = E <= 2;
    constexpr int NS1 = 2 + (QREG ? QCAP : 0);
    __shared__ double sh[NS1 * 64 + 128];            // block_sums_dpp<NS1> | <2> regions (16 waves)
    __shared__ double shq[QREG ? 1 : QCAP * 4 * 16]; // streaming basis dots
    const int done = ctl->done;
    const double n = ctl->n_total, lam = ctl->damping, th = ctl->resth;
    const int maxiter = ctl->maxiter;
    const CgSt sin = *st_in;
    double pv[E], zv[E], xv[E], rv[E];
    int vm[VPACK_PER_THREAD];
    if (vlen) load_vmap(vmap, vlen, vm);
    // every load unconditional (clamped index, value selected after): a load guarded by a run-time
    // condition makes hipcc branch around it and drain vmcnt, serialising the round trips
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int q = threadIdx.x + e * 1024, qc = min(q, P - 1), qw = min(q, nw - 1);
        const bool in = q < P;
        const double p0 = p_in[qc], x0 = x[qc], r0 = r_in[qc];
        double za[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) za[k] = acc[(long)min(k, R_in - 1) * Ps + qw];
        double z = za[0];                              // the summation order of the guarded form
#pragma unroll
        for (int k = 1; k < 8; ++k) z += k < R_in ? za[k] : 0.0;
        pv[e] = in ? p0 : 0.0;
        xv[e] = in ? x0 : 0.0;
        rv[e] = in ? r0 : 0.0;
        zv[e] = q < nw ? z : 0.0;
    }
    [[maybe_unused]] double qv[QREG ? QCAP : 1][E];
    if constexpr (QREG) {
        // qbuf == nullptr (no reorthogonalisation, or the LAST step of a solve -- whose r', p' nobody
        // reads): no basis loads at all (a kernel-argument-uniform branch)
        if (qbuf) {
#pragma unroll
            for (int i = 0; i < QCAP; ++i) qload<E>(qv[i], qbuf, qz, P, Ps, i, nq, 1024);
        } else {
#pragma unroll
            for (int i = 0; i < QCAP; ++i)
#pragma unroll
                for (int e = 0; e < E; ++e) qv[i][e] = 0.0;
        }
    }
    if (done) {
        for (int e = threadIdx.x; e < zero_len; e += 1024) acc_zero[e] = 0.0;   // inputs unused
        return;
    }
    double s1[NS1];
#pragma unroll
    for (int k = 0; k < NS1; ++k) s1[k] = 0.0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int q = threadIdx.x + e * 1024;
        zv[e] = (q < nw ? zv[e] / n : 2.0 * pv[e]) + lam * pv[e];
        s1[0] += pv[e] * zv[e];
        s1[1] += rv[e] * zv[e];
        if constexpr (QREG) {
#pragma unroll
            for (int i = 0; i < QCAP; ++i) s1[2 + i] += qv[i][e] * zv[e];
        }
    }
    const bool ro = qbuf != nullptr && sin.rdotr > 0.0;     // residual reorthogonalisation (QCAP)
    if constexpr (!QREG) {
        if (ro && nq > 0) qdots_stage1<E>(qbuf, qz, P, Ps, nq, zv, 1024, shq);
    }
    block_sums_dpp<NS1, 16>(s1, sh);
    const double alpha = sin.rdotr / s1[0];
    const double cr = ro ? (sqrt(sin.rdotr) - alpha * (s1[1] / sqrt(sin.rdotr))) / sqrt(sin.rdotr) : 0.0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const double r0 = rv[e];
        xv[e] += alpha * pv[e];
        rv[e] -= alpha * zv[e];
        rv[e] -= cr * r0;
    }
    double cs = cr * cr * sin.rdotr;                     // the removed components, squared (ctl->orth)
    if constexpr (QREG) {
        if (ro) {
#pragma unroll
            for (int i = 0; i < QCAP; ++i) {
                const double c = -alpha * s1[2 + i];         // zero for the slots >= nq
                cs += c * c;
#pragma unroll
                for (int e = 0; e < E; ++e) rv[e] -= c * qv[i][e];
            }
        }
    } else {
        if (ro && nq > 0) cs += qcorrect<E>(qbuf, qz, P, Ps, nq, 1024, shq, alpha, rv);
    }
    double rr = 0.0, xx = 0.0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        rr += rv[e] * rv[e];
        xx += xv[e] * xv[e];
    }
    double s2[2] = {rr, xx};
    block_sums_dpp<2, 16>(s2, sh + NS1 * 64);
    const double nr = s2[0], xn = s2[1];
    const double beta = nr / sin.rdotr;
    extern __shared__ double sp[];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int q = threadIdx.x + e * 1024;
        if (q < P) {
            const double pn = rv[e] + beta * pv[e];
            x[q] = xv[e];
            if (r_out) {                               // nullptr: the last step (only x is read)
                r_out[q] = rv[e];
                p_out[q] = pn;
            }
            if (vlen) sp[q] = pn;
        }
    }
    if (vlen) {                                        // fp32 fragment pack of p' for the next FVP
        __syncthreads();
        write_vpack(sp, vm, vpack, vlen, f64);
    }
    qstore<E>(qbuf, P, Ps, sin.iter + 1, nr, rv, 1024);
    if (threadIdx.x == 0) {
        const int it = sin.iter + 1;
        st_out->rdotr = nr;
        st_out->xx = xn;
        st_out->iter = it;
        ctl->iter = it;
        ctl->rdotr = nr;
        hist[2 * it] = nr;
        hist[2 * it + 1] = sqrt(xn);
        ctl->done = (nr < th || it >= maxiter) ? 1 : 0;
        if (ro) note_orth(&ctl->orth, cs, nr);
        if (it <= CG_AMAX) ctl->alpha[it - 1] = alpha;
    }
    // every thread's reads of acc were consumed before block_sums_dpp's barriers
    for (int e = threadIdx.x; e < zero_len; e += 1024) acc_zero[e] = 0.0;
}

// ---------------------------------------------------------------------------
// Distributed CG step for the large-P paths (cooperative kernel: 2x64 and the fp64 mode), SURVEY §8a
// src/TRPO_CG.c:65-103.  The fused form (every FVP block redoing the step on all P elements, the
// basis streamed twice) re-reads ~(4 + 2 nq) P-vectors per block -- at P = 5 443 that is 0.2-0.6 MB
// per CU per iteration.  Here the step is split over natural-order slices instead:
//   cg_dots_kernel : z = zacc / N + lambda p (log-std block 2p + lambda p) for its slice, and the
//                    slice's partial dots p.z, r.z, z.z, x.p, p.p, q_i.z (i < nq) -> dots (DOTS_AT)
//   cg_axpy_kernel : every block sums the partial dots over the blocks in block order (fixed order:
//                    every block gets the same bits), forms alpha, the reorthogonalisation
//                    coefficients, |r'|^2 and beta as in the fused step, and updates its slice:
//                    x += alpha p, r' = r - alpha z - c_r r - sum_i c_i q_i, p' = r' + beta p, the new
//                    basis vector r' / |r'|; block 0 publishes the scalars and the history.
// The next FVP gathers its direction fragments from p' (natural order).  Elements as adjacent pairs
// (one 16-byte load per vector per thread), CGS_T threads per block.
// ---------------------------------------------------------------------------
// The LAST step of a fused CG solve (src/TRPO_CG.c:65-103 for i = maxiter - 1) for P <= 1024: only x
// is read afterwards, so no basis, no reorthogonalisation and no r' / p' stores.  One 512-thread
// workgroup owns adjacent element pairs (16-byte loads of the replicas, p, r, x: the CG-iteration
// kernel's layout); ONE block reduction of p.z, r.z, z.z, x.p, p.p gives alpha, |r'|^2 = |r|^2 -
// 2a r.z + a^2 z.z and |x'|^2 = |x|^2 + 2a x.p + a^2 p.p (the fused step's expansion; direct = 1 -- the
// fp64 mode -- sums |r'|^2 and |x'|^2 directly in a second reduction instead, as cg_update_kernel).
// Zeroes acc_zero (the next solve's first atomic target) after consuming its input.
constexpr int CGL_T = 512;
__global__ void __launch_bounds__(CGL_T)
cg_last_kernel(const double *__restrict__ acc, int R_in, const double *__restrict__ p_in,
               const double *__restrict__ r_in, double *__restrict__ x, int P, int Ps, int nw, Ctl *ctl,
               const CgSt *st_in, CgSt *st_out, double *hist, double *acc_zero, int zero_len, int direct) {
#pragma clang fp contract(off)
    __shared__ double sh[8 * 4 * (CGL_T / 64)];
    const int tid = threadIdx.x;
    const int done = ctl->done;
    const double n = ctl->n_total, lam = ctl->damping, th = ctl->resth;
    const int maxiter = ctl->maxiter;
    const CgSt sin = *st_in;
    const double2 p2 = pair_at(p_in, 0, Ps), r2 = pair_at(r_in, 0, Ps), x2 = pair_at(x, 0, Ps);
    double2 za[RMAX];
#pragma unroll
    for (int k = 0; k < RMAX; ++k) za[k] = pair_at(acc, min(k, R_in - 1), Ps);
    // every loaded value pinned in registers BEFORE the done test: z is only used for q < nw, and with
    // the fp64 division behind it hipcc turned that select into a branch and sank half the replica loads
    // into it (a second round trip, round 5); and with the pins after the done test it sank all of them
    // below that test, behind the ctl->done load (a third round trip: kernel arguments, ctl, vectors)
    double zr[2][RMAX];
#pragma unroll
    for (int k = 0; k < RMAX; ++k) {
        zr[0][k] = za[k].x;
        zr[1][k] = za[k].y;
        asm volatile("" : "+v"(zr[0][k]), "+v"(zr[1][k]));
    }
    double pe[2] = {p2.x, p2.y}, re[2] = {r2.x, r2.y}, xe[2] = {x2.x, x2.y};
    asm volatile("" : "+v"(pe[0]), "+v"(pe[1]), "+v"(re[0]), "+v"(re[1]), "+v"(xe[0]), "+v"(xe[1]));
    if (done) {
        for (int e = tid; e < zero_len; e += CGL_T) acc_zero[e] = 0.0;   // inputs unused
        return;
    }
    double pv[2], rv[2], xv[2], zv[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const int q = 2 * tid + e;
        const bool in = q < P;
        double z = zr[e][0];
#pragma unroll
        for (int k = 1; k < RMAX; ++k) z += k < R_in ? zr[e][k] : 0.0;
        pv[e] = in ? pe[e] : 0.0;
        rv[e] = in ? re[e] : 0.0;
        xv[e] = in ? xe[e] : 0.0;
        zv[e] = in ? __builtin_fma(lam, pv[e], q < nw ? z / n : 2.0 * pv[e]) : 0.0;
    }
    double red[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        red[0] = __builtin_fma(pv[e], zv[e], red[0]);
        red[1] = __builtin_fma(rv[e], zv[e], red[1]);
        red[2] = __builtin_fma(zv[e], zv[e], red[2]);
        red[3] = __builtin_fma(xv[e], pv[e], red[3]);
        red[4] = __builtin_fma(pv[e], pv[e], red[4]);
    }
    block_sums_dpp<5, CGL_T / 64>(red, sh);
    const double alpha = sin.rdotr / red[0];
    double nr = sin.rdotr - 2.0 * alpha * red[1] + alpha * alpha * red[2];
    double xn2 = sin.xx + 2.0 * alpha * red[3] + alpha * alpha * red[4];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        xv[e] = __builtin_fma(alpha, pv[e], xv[e]);
        rv[e] = __builtin_fma(-alpha, zv[e], rv[e]);
    }
    if (direct) {                                       // kernel-argument-uniform
        double s2[2] = {rv[0] * rv[0] + rv[1] * rv[1], xv[0] * xv[0] + xv[1] * xv[1]};
        block_sums_dpp<2, CGL_T / 64>(s2, sh + 5 * 4 * (CGL_T / 64));
        nr = s2[0];
        xn2 = s2[1];
    }
    if (2 * tid + 1 < P) {
        reinterpret_cast<double2 *>(x)[tid] = make_double2(xv[0], xv[1]);
    } else if (2 * tid < P) {
        x[2 * tid] = xv[0];
    }
    if (tid == 0) {
        const int it = sin.iter + 1;
        st_out->rdotr = nr;
        st_out->xx = xn2;
        st_out->iter = it;
        ctl->iter = it;
        ctl->rdotr = nr;
        hist[2 * it] = nr;
        hist[2 * it + 1] = sqrt(xn2);
        ctl->done = (nr < th || it >= maxiter) ? 1 : 0;
        if (it <= CG_AMAX) ctl->alpha[it - 1] = alpha;
    }
    // every thread's reads of acc were consumed before the block reduction's barrier
    for (int e = tid; e < zero_len; e += CGL_T) acc_zero[e] = 0.0;
}

constexpr int CGS_T = 256, CGS_K = 5 + QCAP;
// layout of the per-block partial dots (value k of block b of G): block-major [b][CGS_K] (default) or
// value-major [k][G] (TRPO_DOTS_VMAJ=1: cg_axpy's loads coalesced, but each producer block's 21 values
// land on 21 lines shared with other blocks)
#define DOTS_AT(k, b, G) ((long)(b) * CGS_K + (k))
template <typename QT>
__global__ void __launch_bounds__(CGS_T)
cg_dots_kernel(const double *__restrict__ zacc, const double *__restrict__ p, const double *__restrict__ r,
               const double *__restrict__ x, double *__restrict__ zbuf, double *__restrict__ dots, const void *qbuf_v,
               const void *qz_v, int nq, int P, int Ps, int nw, const Ctl *__restrict__ ctl, const int *__restrict__ skip) {
#pragma clang fp contract(off)
    __shared__ double sh[CGS_K > 16 ? 32 * (CGS_T / 64) : 16 * (CGS_T / 64)];
    const QT *Q = reinterpret_cast<const QT *>(qbuf_v);
    const QT *qz = reinterpret_cast<const QT *>(qz_v);
    const int tid = threadIdx.x, t = blockIdx.x * CGS_T + tid;        // pair index
    const int tc = min(t, (Ps >> 1) - 1);
    const double2 p2 = reinterpret_cast<const double2 *>(p)[tc], r2 = reinterpret_cast<const double2 *>(r)[tc];
    const double2 x2 = reinterpret_cast<const double2 *>(x)[tc], a2 = reinterpret_cast<const double2 *>(zacc)[tc];
    double qv[QCAP][2];
    typedef typename V2T<QT>::type QV2;
#pragma unroll
    for (int i = 0; i < QCAP; ++i) {
        const bool ok = i < nq;
        const QV2 *src = ok ? reinterpret_cast<const QV2 *>(Q + (long)i * Ps) + tc
                            : reinterpret_cast<const QV2 *>(qz) + (tid & 7);
        const QV2 v = *src;
        qv[i][0] = ok ? (double)v.x : 0.0;
        qv[i][1] = ok ? (double)v.y : 0.0;
    }
    const double cn = ctl->n_total, lam = ctl->damping;
    if (*skip) return;                                    // grid-uniform
    const double pe[2] = {p2.x, p2.y}, re[2] = {r2.x, r2.y}, xe[2] = {x2.x, x2.y}, ae[2] = {a2.x, a2.y};
    double red[CGS_K];
#pragma unroll
    for (int k = 0; k < CGS_K; ++k) red[k] = 0.0;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const int q = 2 * t + e;
        const bool in = q < P;
        const double pv = in ? pe[e] : 0.0, rv = in ? re[e] : 0.0, xv = in ? xe[e] : 0.0;
        const double zv = in ? __builtin_fma(lam, pv, q < nw ? ae[e] / cn : 2.0 * pv) : 0.0;
        if (in) zbuf[q] = zv;
        red[0] = __builtin_fma(pv, zv, red[0]);
        red[1] = __builtin_fma(rv, zv, red[1]);
        red[2] = __builtin_fma(zv, zv, red[2]);
        red[3] = __builtin_fma(xv, pv, red[3]);
        red[4] = __builtin_fma(pv, pv, red[4]);
#pragma unroll
        for (int i = 0; i < QCAP; ++i) red[5 + i] = __builtin_fma(in ? qv[i][e] : 0.0, zv, red[5 + i]);
    }
    block_sums_dpp<CGS_K, CGS_T / 64>(red, sh);
    if (tid < CGS_K) {
        double v = red[0];
#pragma unroll
        for (int k = 1; k < CGS_K; ++k) v = tid == k ? red[k] : v;
        dots[DOTS_AT(tid, blockIdx.x, gridDim.x)] = v;
    }
}

// The CG step over natural-order slices (src/TRPO_CG.c:77-103 with the reorthogonalisation of DESIGN §3):
// slice `sl` (CGS_T pairs) of x, r, p, the basis vector q_it and the fp32 direction pack, from the G producer
// blocks' partial dots.  Two phases, so that a caller can issue the loads of the step's inputs (p, r, x,
// the pack slots, the basis -- none of them written by the producers) before it waits for the producers:
// axpy_load_inputs, then axpy_finish (z and the partial dots, the step, the stores).
template <typename QT> struct AxIn {
    double2 p2, r2, x2;
    int2 ps2;
    double qv[QCAP][2];
};
template <typename QT>
__device__ __forceinline__ void axpy_load_inputs(AxIn<QT> &in, int sl, const double *__restrict__ p_in,
                                                 const double *__restrict__ r_in, const double *__restrict__ x,
                                                 const void *qbuf_v, const void *qz_v, int nq, int Ps,
                                                 const float *vpk, const int *__restrict__ pslot) {
    const QT *Q = reinterpret_cast<const QT *>(qbuf_v);
    const QT *qz = reinterpret_cast<const QT *>(qz_v);
    const int tid = threadIdx.x, t = sl * CGS_T + tid;
    const int tc = min(t, (Ps >> 1) - 1);
    in.p2 = reinterpret_cast<const double2 *>(p_in)[tc];
    in.r2 = reinterpret_cast<const double2 *>(r_in)[tc];
    in.x2 = reinterpret_cast<const double2 *>(x)[tc];
    // vpk: p' also into the fp32 fragment-order direction pack of the next FVP (slots pslot[q], -1 for
    // LogStd), so its cooperative kernel loads the pack coalesced instead of gathering p' itself
    in.ps2 = vpk ? reinterpret_cast<const int2 *>(pslot)[tc] : make_int2(-1, -1);
    typedef typename V2T<QT>::type QV2;
#pragma unroll
    for (int i = 0; i < QCAP; ++i) {
        const bool ok = i < nq;
        const QV2 *src = ok ? reinterpret_cast<const QV2 *>(Q + (long)i * Ps) + tc
                            : reinterpret_cast<const QV2 *>(qz) + (tid & 7);
        const QV2 v = *src;
        in.qv[i][0] = ok ? (double)v.x : 0.0;
        in.qv[i][1] = ok ? (double)v.y : 0.0;
    }
}
template <typename QT>
__device__ __forceinline__ void axpy_finish(const AxIn<QT> &in, int sl, const double *__restrict__ dots, int G,
                                            const double *__restrict__ zbuf, double *__restrict__ p_out,
                                            double *__restrict__ r_out, double *__restrict__ x, void *qbuf_v,
                                            int reorth, int P, int Ps, Ctl *__restrict__ ctl,
                                            const CgSt *__restrict__ st_in, CgSt *__restrict__ st_out,
                                            double *__restrict__ hist, float *__restrict__ vpk, double *tot) {
#pragma clang fp contract(off)
    QT *Q = reinterpret_cast<QT *>(qbuf_v);
    const int tid = threadIdx.x, t = sl * CGS_T + tid;
    const int tc = min(t, (Ps >> 1) - 1);
    const double2 z2 = reinterpret_cast<const double2 *>(zbuf)[tc];
    // the partial dots of the G producer blocks (DOTS_AT): wave w sums values k = w,
    // w + 4, ...; lane l takes partials l, l + 64, l + 128, l + 192 (all loads issued together, unconditional), then the
    // fixed-order wave tree (a serial chain of G dependent loads by one thread was measured ~100 us
    // at G = 176 partials)
    constexpr int NW = CGS_T / 64, NI = (CGS_K + NW - 1) / NW, NJ = 4;
    const int lane = tid & 63, w = tid >> 6;
    double pv_[NI];
    {
        double v[NI][NJ];
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int k = w + NW * i, b = lane + 64 * j;
                const double d = dots[DOTS_AT(min(k, CGS_K - 1), min(b, G - 1), G)];
                // a multiply, not a select: with `cond ? d : 0` hipcc sank the loads under the condition
                // (exec-masked, one vmcnt(0) drain each: 16 serialised round trips, round 5)
                v[i][j] = d * ((k < CGS_K && b < G) ? 1.0 : 0.0);
            }
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            double a = (v[i][0] + v[i][1]) + (v[i][2] + v[i][3]);
            for (int b = lane + 64 * NJ; b < G; b += 64) a += dots[DOTS_AT(min(w + NW * i, CGS_K - 1), b, G)];
            pv_[i] = wave_tree_sum(a);
        }
    }
    const CgSt sin = *st_in;
    const double cth = ctl->resth;
    const int cmax = ctl->maxiter;
    // grid-uniform stop test on the state this step starts from: the value ctl->done held when the
    // launch began (cg_init_kernel / the previous step set it by this formula).  Not *skip: block 0
    // of THIS launch rewrites ctl->done at its end, and a block that starts after that (a GPU shared
    // with other processes) would skip its slice of the final x update.  A stopped step carries the
    // state forward (st_out = st_in) so that the next launch's test sees it too.
    if (sin.rdotr < cth || sin.iter >= cmax) {
        if (sl == 0 && tid == 0) *st_out = sin;
        return;
    }
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < NI; ++i)
            if (w + NW * i < CGS_K) tot[w + NW * i] = pv_[i];
    }
    __syncthreads();
    const double pz = tot[0], rz = tot[1], zz = tot[2], xp = tot[3], pp = tot[4];
    const double alpha = sin.rdotr / pz;
    // reorthogonalisation coefficients (as the fused step, fvp_mlp3_kernel / DESIGN §3)
    double cs = 0.0, cr = 0.0;
    const bool ro = reorth && sin.rdotr > 0.0;
    if (ro) {
        const double nrm = sqrt(sin.rdotr), cl = nrm - alpha * (rz / nrm);
        cs = cl * cl;
        cr = cl / nrm;
    }
    double c[QCAP];
#pragma unroll
    for (int i = 0; i < QCAP; ++i) {
        c[i] = ro ? -alpha * tot[5 + i] : 0.0;             // zero for the slots >= nq
        cs += c[i] * c[i];
    }
    const double nr = sin.rdotr - 2.0 * alpha * rz + alpha * alpha * zz - cs;
    const double xn2 = sin.xx + 2.0 * alpha * xp + alpha * alpha * pp;
    const double beta = nr / sin.rdotr;
    const int it = sin.iter + 1;
    const double pe[2] = {in.p2.x, in.p2.y}, re[2] = {in.r2.x, in.r2.y}, xe[2] = {in.x2.x, in.x2.y},
                 ze[2] = {z2.x, z2.y};
    double xo[2], ro2[2], po[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        double rv = __builtin_fma(-alpha, ze[e], re[e]);
        rv = __builtin_fma(-cr, re[e], rv);
#pragma unroll
        for (int i = 0; i < QCAP; ++i) rv = __builtin_fma(-c[i], in.qv[i][e], rv);
        ro2[e] = rv;
        xo[e] = __builtin_fma(alpha, pe[e], xe[e]);
        po[e] = __builtin_fma(beta, pe[e], rv);
    }
    if (2 * t + 1 < P) {                                 // whole pairs: 16-byte stores
        reinterpret_cast<double2 *>(x)[t] = make_double2(xo[0], xo[1]);
        reinterpret_cast<double2 *>(r_out)[t] = make_double2(ro2[0], ro2[1]);
        reinterpret_cast<double2 *>(p_out)[t] = make_double2(po[0], po[1]);
    } else if (2 * t < P) {
        x[2 * t] = xo[0];
        r_out[2 * t] = ro2[0];
        p_out[2 * t] = po[0];
    }
    if (vpk) {
        if (2 * t < P && in.ps2.x >= 0) vpk[in.ps2.x] = (float)po[0];
        if (2 * t + 1 < P && in.ps2.y >= 0) vpk[in.ps2.y] = (float)po[1];
    }
    if (reorth && it < QCAP) {                            // q_it = r' / |r'|
        const double inv = nr > 0.0 ? 1.0 / sqrt(nr) : 0.0;
#pragma unroll
        for (int e = 0; e < 2; ++e)
            if (2 * t + e < P) Q[(long)it * Ps + 2 * t + e] = (QT)(ro2[e] * inv);
    }
    if (sl == 0 && tid == 0) {
        const int done = (nr < cth || it >= cmax) ? 1 : 0;
        st_out->rdotr = nr;
        st_out->xx = xn2;
        st_out->iter = it;
        hist[2 * it] = nr;
        hist[2 * it + 1] = sqrt(xn2);
        ctl->rdotr = nr;
        ctl->iter = it;
        ctl->done = done;
        note_orth(&ctl->orth, cs, nr);
        if (it <= CG_AMAX) ctl->alpha[it - 1] = alpha;
    }
}

template <typename QT>
__global__ void __launch_bounds__(CGS_T)
cg_axpy_kernel(const double *__restrict__ dots, int G, const double *__restrict__ zbuf,
               const double *__restrict__ p_in, const double *__restrict__ r_in, double *__restrict__ p_out,
               double *__restrict__ r_out, double *__restrict__ x, void *qbuf_v, const void *qz_v, int nq, int reorth,
               int P, int Ps, Ctl *__restrict__ ctl, const CgSt *__restrict__ st_in, CgSt *__restrict__ st_out,
               double *__restrict__ hist, const int *__restrict__ skip, float *__restrict__ vpk = nullptr,
               const int *__restrict__ pslot = nullptr) {
    __shared__ double tot[CGS_K];
    (void)skip;
    AxIn<QT> in;
    axpy_load_inputs<QT>(in, blockIdx.x, p_in, r_in, x, qbuf_v, qz_v, nq, Ps, vpk, pslot);
    axpy_finish<QT>(in, blockIdx.x, dots, G, zbuf, p_out, r_out, x, qbuf_v, reorth, P, Ps, ctl, st_in, st_out, hist, vpk,
                    tot);
}

// One rank (no all-reduce between the slab reduce and the step): reduce_slabs_kernel<float> and
// cg_dots_kernel in ONE launch (round 5; TRPO_COOP_RDOTS=0 keeps the two).  Block b reduces its RS_POS
// slab positions exactly as reduce_slabs_kernel does (same loads, same fixed order, the same zacc
// bits), then its threads t < RS_POS that hold a parameter (m = imap[.] >= 0) and, in block 0, the
// threads RS_POS + k (k < P - nw) that hold the log-std entries form z = a / N + lambda p (2p + lambda p)
// as cg_dots_kernel does, store it to zbuf and contribute the partial dots p.z, r.z, z.z, x.p, p.p,
// q_i.z -> dots (DOTS_AT; cg_axpy_kernel sums the slab/RS_POS partials in block order).  The gathers
// of p, r, x and the basis at the block's natural indices are issued between the slab loads and
// their sums, so they add no round trip.  Only the dots' partition differs from the two-kernel form.
// (Round 6, VERDICT r05 #5, measured and dropped: the step itself in this launch -- cg_axpy_kernel's work by
// the first GA blocks once every block had published its z slice and dots, behind eight per-XCD arrival
// counters, the step inputs' loads issued before the wait.  Bit-identical, but the fused launch took 11.6 us
// against 5.3 + 5.4 us for the two, and the 2x64 CG solve 381.0 -> 392.8 us at 50k, 194.4 -> 205.3 us at
// 4 096: the in-kernel fan-in costs more than the launch boundary it removes; profiles/r06_axf_ab.log.)
template <typename QT>
__global__ void __launch_bounds__(RS_THREADS)
reduce_dots_kernel(const float *__restrict__ slabs, int G, int slab, const int *__restrict__ imap,
                   double *__restrict__ zacc, const double *__restrict__ p, const double *__restrict__ r,
                   const double *x, double *__restrict__ zbuf, double *__restrict__ dots,
                   const void *qbuf_v, const void *qz_v, int nq, int P, int Ps, int nw,
                   const Ctl *ctl, const int *__restrict__ skip) {
#pragma clang fp contract(off)
    constexpr int VE = 4, LP = RS_POS / VE, SG = RS_THREADS / LP, NLD = 256 / SG;
    typedef float VT __attribute__((ext_vector_type(VE)));
    __shared__ double part[SG][RS_POS + 1];
    __shared__ double sh[32 * (RS_THREADS / 64)];
    const QT *Q = reinterpret_cast<const QT *>(qbuf_v);
    const QT *qz = reinterpret_cast<const QT *>(qz_v);
    const int t = threadIdx.x, lp = t % LP, sg = t / LP;
    const int j0 = blockIdx.x * RS_POS + lp * VE;
    const int m = t < RS_POS ? imap[blockIdx.x * RS_POS + t] : -1;
    // this thread's parameter: a slab position's, a log-std entry (block 0), or none (-1)
    const int kls = t - RS_POS;
    if (*skip) return;                                    // grid-uniform
    VT v[NLD];
#pragma unroll
    for (int k = 0; k < NLD; ++k) {                       // the first load round (all of it for G <= 256)
        // clamped and masked by a multiply (+-0 adds nothing): a `b < G ? load : 0` became exec-masked
        // loads the compiler cannot count, so it drained them all (vmcnt(0)) before the gathers below
        const int b = sg + SG * k;
        v[k] = *reinterpret_cast<const VT *>(slabs + (long)min(b, G - 1) * slab + j0) * (b < G ? 1.0f : 0.0f);
    }
    const int q = t < RS_POS ? m : (blockIdx.x == 0 && kls >= 0 && kls < P - nw ? nw + kls : -1);
    const int qc = min(max(q, 0), P - 1);
    const double p0 = p[qc], r0 = r[qc], x0 = x[qc];
    double qv[QCAP];
#pragma unroll
    for (int i = 0; i < QCAP; ++i) {
        const bool ok = i < nq;
        const QT qq = ok ? Q[(long)i * Ps + qc] : qz[t & 7];
        qv[i] = ok ? (double)qq : 0.0;
    }
    double s[VE];
#pragma unroll
    for (int e = 0; e < VE; ++e) s[e] = 0.0;
#pragma unroll
    for (int k = 0; k < NLD; ++k)
#pragma unroll
        for (int e = 0; e < VE; ++e) s[e] += (double)v[k][e];
    for (int b0 = sg + SG * NLD; b0 < G; b0 += SG * NLD) {   // G > 256 block partials
#pragma unroll
        for (int k = 0; k < NLD; ++k) {
            const int b = b0 + SG * k;
            v[k] = b < G ? *reinterpret_cast<const VT *>(slabs + (long)b * slab + j0) : (VT)0;
        }
#pragma unroll
        for (int k = 0; k < NLD; ++k)
#pragma unroll
            for (int e = 0; e < VE; ++e) s[e] += (double)v[k][e];
    }
#pragma unroll
    for (int e = 0; e < VE; ++e) part[sg][lp * VE + e] = s[e];
    __syncthreads();
    double a = 0.0;
    if (t < RS_POS) {
#pragma unroll 8
        for (int k = 0; k < SG; ++k) a += part[k][t];
        if (m >= 0) zacc[m] = a;
    }
    const double cn = ctl->n_total, lam = ctl->damping;
    double red[CGS_K];
#pragma unroll
    for (int k = 0; k < CGS_K; ++k) red[k] = 0.0;
    if (q >= 0) {
        const double zv = __builtin_fma(lam, p0, q < nw ? a / cn : 2.0 * p0);
        zbuf[q] = zv;
        red[0] = p0 * zv;
        red[1] = r0 * zv;
        red[2] = zv * zv;
        red[3] = x0 * p0;
        red[4] = p0 * p0;
#pragma unroll
        for (int i = 0; i < QCAP; ++i) red[5 + i] = qv[i] * zv;
    }
    block_sums_dpp<CGS_K, RS_THREADS / 64>(red, sh);
    if (t < CGS_K) {
        double o = red[0];
#pragma unroll
        for (int k = 1; k < CGS_K; ++k) o = t == k ? red[k] : o;
        dots[DOTS_AT(t, blockIdx.x, gridDim.x)] = o;
    }
}

// ===========================================================================
// device layer (trpo_dev.h)
// ===========================================================================
typedef void (*fast_launch_fn)(dim3, int, hipStream_t, const IterArgs &, const Net &);

template <int T0, int T1, int T2, int T3, int ACT, int MODE, int QB = 0, int NO = 0>
static void fast_launch(dim3 g, int lds, hipStream_t st, const IterArgs &a, const Net &net) {
    const int meta = (a.Ps & 0xFFFFF) | ((a.R_in & 63) << 20) | ((a.nq & 63) << 26);
    hipLaunchKernelGGL((fvp_mlp3_kernel<T0, T1, T2, T3, ACT, MODE, QB, NO>), g, dim3(64 * FastCfg<T0, T1, T2, T3>::WAVES),
                       lds, st, a.acc_in, a.p_in, a.r_in, a.x, a.pslot, (const void *)a.q, meta, a, net);
}
// MODE 3 kernels by the reorthogonalisation basis they load in their prologue (QB slots)
constexpr int kQB[4] = {0, 4, 8, QCAP};
static int qb_index(int nq) { return nq <= 0 ? 0 : nq <= 4 ? 1 : nq <= 8 ? 2 : 3; }

// CG kernels are templated on the per-thread element count E = ceil(P / 1024)
static int cg_E(int P) {
    const int e = (P + 1023) / 1024;
    return e <= 1 ? 1 : e <= 2 ? 2 : e <= 4 ? 4 : e <= 8 ? 8 : e <= 16 ? 16 : 32;
}
// QT: the reorthogonalisation basis element type of the context (qbuf_t)
#define CG_DISPATCH_T(E, QT, KERNEL, ...)                                             \
    switch (E) {                                                                      \
    case 1: hipLaunchKernelGGL((KERNEL<1, QT>), __VA_ARGS__); break;                  \
    case 2: hipLaunchKernelGGL((KERNEL<2, QT>), __VA_ARGS__); break;                  \
    case 4: hipLaunchKernelGGL((KERNEL<4, QT>), __VA_ARGS__); break;                  \
    case 8: hipLaunchKernelGGL((KERNEL<8, QT>), __VA_ARGS__); break;                  \
    case 16: hipLaunchKernelGGL((KERNEL<16, QT>), __VA_ARGS__); break;                \
    default: hipLaunchKernelGGL((KERNEL<32, QT>), __VA_ARGS__); break;                \
    }
#define CG_DISPATCH(E, KERNEL, ...)                                                   \
    do {                                                                              \
        if (d->f64) CG_DISPATCH_T(E, double, KERNEL, __VA_ARGS__)                     \
        else CG_DISPATCH_T(E, float, KERNEL, __VA_ARGS__)                             \
    } while (0)
template <int T0, int T1, int T2, int T3, int ACT, int NO = 0>
static hipError_t fast_attr(int lds) {
    hipError_t e = hipFuncSetAttribute((const void *)fvp_mlp3_kernel<T0, T1, T2, T3, ACT, 0, 0, NO>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    if constexpr (FastCfg<T0, T1, T2, T3>::REGW) {
        e = hipFuncSetAttribute((const void *)fvp_mlp3_kernel<T0, T1, T2, T3, ACT, 2, 0, NO>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        if (e != hipSuccess) return e;
        const void *k3[4] = {(const void *)fvp_mlp3_kernel<T0, T1, T2, T3, ACT, 3, kQB[0], NO>,
                             (const void *)fvp_mlp3_kernel<T0, T1, T2, T3, ACT, 3, kQB[1], NO>,
                             (const void *)fvp_mlp3_kernel<T0, T1, T2, T3, ACT, 3, kQB[2], NO>,
                             (const void *)fvp_mlp3_kernel<T0, T1, T2, T3, ACT, 3, kQB[3], NO>};
        for (const void *k : k3) {
            e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
            if (e != hipSuccess) return e;
        }
    }
    return hipFuncSetAttribute((const void *)fvp_mlp3_kernel<T0, T1, T2, T3, ACT, 1, 0, NO>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, lds);
}

// MODE 2 (forward cache) exists for the register-resident small-net shapes only
template <int T0, int T1, int T2, int T3, int ACT, int MODE, int QB = 0, int NO = 0>
static constexpr fast_launch_fn yc_launch() {
    if constexpr (FastCfg<T0, T1, T2, T3>::REGW) return fast_launch<T0, T1, T2, T3, ACT, MODE, QB, NO>;
    else return nullptr;
}

struct FastEntry {
    int T[4];
    int act;                     // -1: run-time activations
    int no;                      // narrow output layer, the kernels' NO (0: 16x16x4 output layer)
    fast_launch_fn launch;
    fast_launch_fn launch_pg;    // MODE 1: policy gradient
    fast_launch_fn launch_yc;    // MODE 2: FVP on the cached forward activations
    fast_launch_fn launch_yc_cg[4]; // MODE 3: the same inside the CG graph, by reorthogonalisation slots kQB
    hipError_t (*attr)(int);
    int lds, tlen, vlen, slab, emax, waves;
};

#define ACT_TTL (ACT_T | (ACT_T << 2) | (ACT_L << 4))
#define FAST_ENTRY_NO(a, b, c, d, act, no)                                                                        \
    {{a, b, c, d}, act, no, fast_launch<a, b, c, d, act, 0, 0, no>, fast_launch<a, b, c, d, act, 1, 0, no>,       \
     yc_launch<a, b, c, d, act, 2, 0, no>(),                                                                      \
     {yc_launch<a, b, c, d, act, 3, kQB[0], no>(), yc_launch<a, b, c, d, act, 3, kQB[1], no>(),                   \
      yc_launch<a, b, c, d, act, 3, kQB[2], no>(), yc_launch<a, b, c, d, act, 3, kQB[3], no>()},                  \
     fast_attr<a, b, c, d, act, no>,                                                                              \
     FastCfg<a, b, c, d>::lds_bytes(), FastCfg<a, b, c, d>::TLEN, FastCfg<a, b, c, d>::VLEN,                      \
     FastCfg<a, b, c, d>::SLAB, FastCfg<a, b, c, d>::EMAX, FastCfg<a, b, c, d>::WAVES}
#define FAST_ENTRY(a, b, c, d, act) FAST_ENTRY_NO(a, b, c, d, act, 0)
#define FAST_SHAPE(a, b, c, d) FAST_ENTRY(a, b, c, d, ACT_TTL), FAST_ENTRY(a, b, c, d, -1)
// narrow output layer (<= 3 or <= 4 outputs; VALU or MFMA RGW2) of the register-resident small-net shape
#define FAST_NO_PAIR(a, b, c, d, act, no) FAST_ENTRY_NO(a, b, c, d, act, no), FAST_ENTRY_NO(a, b, c, d, act, no | NO_MFMA_RGW2)
#define FAST_SHAPE_NO(a, b, c, d)                                                                                 \
    FAST_NO_PAIR(a, b, c, d, ACT_TTL, 3), FAST_NO_PAIR(a, b, c, d, -1, 3), FAST_NO_PAIR(a, b, c, d, ACT_TTL, 4),   \
        FAST_NO_PAIR(a, b, c, d, -1, 4)

static const FastEntry kFast[] = {
    FAST_SHAPE(1, 1, 1, 1), FAST_SHAPE(1, 2, 2, 1), FAST_SHAPE(1, 4, 4, 1),
    FAST_SHAPE(2, 1, 1, 1), FAST_SHAPE(2, 2, 2, 1), FAST_SHAPE(2, 4, 4, 1),
    FAST_SHAPE_NO(1, 1, 1, 1),
};

// cooperative kernels (T1 == T2 == TH, T3 == 1); element type T: fp32 or the fp64 precision mode;
// NO: the narrow output layer (fp32, <= 4 outputs)
template <typename T, int T0, int TH, int ACT, int MODE, int NO = 0>
static void coop_launch(dim3 g, int lds, hipStream_t st, const IterArgs &a, const Net &net) {
    hipLaunchKernelGGL((fvp_coop_kernel<T, T0, TH, ACT, MODE, NO>), g, dim3(CoopCfg<T, T0, TH>::THREADS), lds, st,
                       a, net);
}
template <typename T, int T0, int TH>
struct CoopYC {
    static constexpr bool ok = sizeof(T) == 4 ? !(T0 == 2 && TH == 4) : true;
};
template <typename T, int T0, int TH, int ACT, int NO = 0>
static hipError_t coop_attr(int lds) {
    const void *k[5] = {(const void *)fvp_coop_kernel<T, T0, TH, ACT, 0, NO>,
                        (const void *)fvp_coop_kernel<T, T0, TH, ACT, 1, NO>,
                        (const void *)fvp_coop_kernel<T, T0, TH, ACT, 2, NO>, nullptr, nullptr};
    if constexpr (CoopYC<T, T0, TH>::ok) {
        k[3] = (const void *)fvp_coop_kernel<T, T0, TH, ACT, 3, NO>;
        k[4] = (const void *)fvp_coop_kernel<T, T0, TH, ACT, 4, NO>;
    }
    for (const void *f : k) {
        if (!f) continue;
        const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}
// MODE 3 / 4 (forward cache): not where the cache registers push the kernel into scratch spills
// (fp32 T0 = 2, TH = 4; fp64 TH = 1, whose 8-wave blocks cap a wave at 256 VGPRs)
template <typename T, int T0, int TH, int ACT, int MODE, int NO = 0>
static constexpr fast_launch_fn coop_yc_launch() {
    if constexpr (CoopYC<T, T0, TH>::ok) return coop_launch<T, T0, TH, ACT, MODE, NO>;
    else return nullptr;
}
struct CoopEntry {
    int f64, T0, TH, act, no;
    fast_launch_fn launch, launch_pg, launch_cg;   // MODE 0 FVP, 1 policy gradient, 2 CG iteration
    fast_launch_fn launch_yc, launch_cg_yc;        // MODE 3 / 4: 0 / 2 on the forward cache (fp32)
    hipError_t (*attr)(int);
    int lds, slab, ng, threads, main_bytes;
};
#define COOP_ENTRY_NO(T, t0, th, act, no)                                                                         \
    {sizeof(T) == 8, t0, th, act, no, coop_launch<T, t0, th, act, 0, no>, coop_launch<T, t0, th, act, 1, no>,     \
     coop_launch<T, t0, th, act, 2, no>, coop_yc_launch<T, t0, th, act, 3, no>(),                                \
     coop_yc_launch<T, t0, th, act, 4, no>(), coop_attr<T, t0, th, act, no>, CoopCfg<T, t0, th>::LDS_BYTES,      \
     CoopSlab<T, t0, th, no>::SLAB, CoopCfg<T, t0, th>::NG, CoopCfg<T, t0, th>::THREADS, CoopCfg<T, t0, th>::MAIN_BYTES}
#define COOP_ENTRY(T, t0, th, act) COOP_ENTRY_NO(T, t0, th, act, 0)
#define COOP_SHAPE(T, t0, th) COOP_ENTRY(T, t0, th, ACT_TTL), COOP_ENTRY(T, t0, th, -1)
#define COOP_SHAPE_NO(t0, th) COOP_ENTRY_NO(float, t0, th, ACT_TTL, 4), COOP_ENTRY_NO(float, t0, th, -1, 4)
static const CoopEntry kCoop[] = {
    COOP_SHAPE(float, 1, 2),  COOP_SHAPE(float, 1, 4),  COOP_SHAPE(float, 2, 2),  COOP_SHAPE(float, 2, 4),
    COOP_SHAPE(double, 1, 1), COOP_SHAPE(double, 1, 2), COOP_SHAPE(double, 1, 4), COOP_SHAPE(double, 2, 1),
    COOP_SHAPE(double, 2, 2), COOP_SHAPE(double, 2, 4),
    COOP_SHAPE_NO(1, 2),      COOP_SHAPE_NO(1, 4),      COOP_SHAPE_NO(2, 2),      COOP_SHAPE_NO(2, 4)};

struct trpo_dev {
    int device;
    hipStream_t stream;
    Net net;
    int P, nw;
    int Ps;                     // even row stride of replica sets and the basis: P rounded up to even
    // fast path
    const FastEntry *fast;
    const FastEntry *fast_no[2];  // narrow-output twins of fast: [0] MFMA RGW2 (few tiles per wave), [1] VALU RGW2
    const CoopEntry *coop_e;    // cooperative kernel for wide hidden layers (else NULL)
    int coop;
    int coop_fused;             // CG step fused into the cooperative FVP kernel (MODE 2)
    int coop_dist;              // cooperative path: the CG step over slices (cg_dots / cg_axpy), TRPO_COOP_DIST
    int coop_pk;                // ... cg_axpy also writes p' into the fp32 direction pack (TRPO_COOP_PK, round 5)
    int coop_rdots;             // ... one rank: slab reduce + dots in one launch (TRPO_COOP_RDOTS, round 5)
    int coop_gmaj;              // cooperative kernel: group-major tile order (TRPO_COOP_GMAJ: 1 on, 0 off, unset auto)
    int gmaj_on;                // ... in effect for the current sample count (choose_grid)
    int gmaj_fvp, grid_fvp;     // ... and the tile order / grid of the standalone FVP calls (choose_grid)
    int vpack_v;                // the fp32 direction pack holds slot V (written by its upload; any other
                                // writer of the pack -- a CG, a gathered FVP -- clears it)
    int cinit;                  // cooperative CG start inside the first FVP launch (TRPO_COOP_CINIT, default 1)
    double *zbuf, *dotsbuf;     // its z (natural order, Ps) and per-block partial dots
    fast_launch_fn k_fvp, k_pg; // the tile kernel serving this shape, FVP and policy-gradient modes
    fast_launch_fn k_fvp_yc, k_cg_yc;   // the same kernel on the forward cache: standalone FVP, CG iteration
    fast_launch_fn k_cg_yc_q[4];        // one-wave-per-tile CG iteration by reorthogonalisation slots (kQB)
    void *qbuf;                         // reorthogonalisation basis QT [QCAP][P] (QT: fp32, fp64 mode fp64)
    double *qzero;                      // a zero line
    int reorth;                         // TRPO_CG_REORTH (default 1)
    int k_lds, k_tiles;         // its dynamic LDS bytes and tiles per block per step
    Pack pack;
    int f64;                    // fp64 precision mode: fp64 packs/observations/slabs, fp64 MFMA kernel
    size_t esz;                 // pack / observation / slab element bytes (4 or 8)
    void *tpack, *vpack;
    int *tmap, *vmap;
    int *pslot;                 // natural parameter -> v-pack slot (-1: LogStd)
    int *islot;                 // natural parameter -> the tile kernel's accumulator position (epilogue)
    int *imap;                  // slab position -> natural parameter (reduce kernel)
    int slab;                   // floats per block partial
    void *obs4;
    // forward-activation cache of the one-wave-per-tile kernel (MODE 0 writes, MODE 2 reads):
    // f4 [ntiles][T1 + T2 + T3][64]; valid for the current theta / observations when yc_valid
    void *yc;
    size_t yc_cap;              // bytes
    int yc_on, yc_valid;
    // generic path
    void *gth, *gv, *giv, *gobs, *scratch;   // generic path: theta, direction, 1/sigma^2, observations (esz)
    int srows;
    size_t scratch_blocks;
    // common
    double *theta64;            // natural theta (device, fp64)
    double *obs64;              // local observations [n][L0], fp64 (TRPO_Update path)
    void *pg_d, *pg_adv, *pg_iv;    // policy-gradient mode inputs (element esz, padded like obs4)
    size_t pg_cap;
    unsigned pg_gen;                // rollout generation pg_d / pg_adv were built from
    size_t pg_n;
    void *upd;                  // TRPO_Update path state (trpo_update.hip)
    double *std64;
    double *vec[5];             // V, Z, X, B, P
    double *r, *zacc;
    double *pbuf[2], *rbuf[2];  // ping-ponged CG direction / residual
    CgSt *st;                   // 2 ping-ponged CG scalar states
    double *accbuf;             // atomic mode: 3 x R fp64 replicas of the P-vector
    double *pacc;               // atomic mode, standalone FVPs: R replicas (set 0; left zeroed by the
                                // epilogue) + a sink set for epilogue-less kernel-only timing launches
    int atomic, R;
    int Rc;                     // replicas in use: R on one GPU; under RCCL sized from the global shard
                                // geometry (identical on every rank) to keep the all-reduce small
    void *slabs;
    int slab_blocks;            // capacity
    int grid;                   // FVP blocks for the current n
    Ctl *ctl;
    double *hist;               // 2 * (maxiter_cap + 1)
    int hist_cap;
    size_t n;                   // local samples
    size_t npad_cap;
    double n_total;
    double n_max;               // largest shard over the ranks (replica sizing)
    double damping;
    // CG graph cache
    hipGraphExec_t cg_exec;
    int no_graph;
    size_t cg_graph_iters;
    double cg_graph_resth;
    size_t cg_last_iters;       // maxiter of the last enqueued CG (trpo_dev_ycache_written)
    void *tscr;                 // scratch of the kernel-only timing of the CG-iteration kernel
    hipEvent_t ev0, ev1;
    // pinned, device-mapped host staging for the host <-> device vector moves (kernel copies)
    double *hst, *hst_dev;
    size_t hst_cap;
    int hst_pending;        // an upload's copy kernel may still read hst: sync before the host rewrites it
    // trpo_dev_wait_done without a collective: a stream write of wseq into this pinned word, then a spin
    unsigned *wflag, *wflag_dev;
    unsigned wseq;
    // RCCL
    ncclComm_t comm;
    // in-process host-staged group (trpo_dev_set_group): the same sharded code path without RCCL
    trpo_hgroup *group;
    double *gbuf, *gbuf_dev;    // pinned (coherent, mapped) host staging for the group exchange
    size_t gbuf_cap;
    // peer-window exchange over xGMI (trpo_peer.hip): when peer_on, every collective goes through it
    // and the CG graph's per-FVP all-reduce becomes one exchange kernel into zred
    trpo_peer *peer;
    int peer_on;
    double *zred;               // [2][Ps] exchanged partial sums (the next CG-iteration kernel's input)
    double *ptmp;               // [slot] staging of an in-place all-reduce
    double *pn;                 // [PEER_WMAX] the shard sizes exchanged at attach
    int rank, world;
    int comm_aborted;           // trpo_dev_comm_abort ran: every later result call reports -4
    int no_cg_last;             // TRPO_CG_LAST=0: the last step on cg_update_kernel (A/B)
    char name[64];
};

// this context's partial sums are one rank's share: every collective backend (RCCL, host group, peer
// windows) counts, so FVP epilogues must wait for allreduce() whenever this holds
static inline bool has_collective(const trpo_dev *d) { return d->comm || d->group || d->peer_on; }

// ---------------------------------------------------------------------------
// In-process host-staged all-reduce (trpo_dev_set_group).  The contexts of one process -- one
// thread per context, on any devices -- exchange their partial sums through host memory: every rank
// copies its buffer in, waits for all ranks, sums the slots in rank order (so every rank gets the
// same bits, as RCCL's all-reduce guarantees) and copies the sum back.  It exists to run the
// library's sharded code path (global N, replica sizing from the largest shard, lockstep CG) on a
// single GPU in tests; the collective is a host round trip, so CG runs eagerly under it.
// ---------------------------------------------------------------------------
struct trpo_hgroup {
    int world;
    pthread_barrier_t bar;
    pthread_mutex_t mu;
    double **slot;              // per-rank host views of the buffers being reduced
    size_t *count;
    int *attached;
};

extern "C" trpo_hgroup *trpo_hgroup_create(int world) {
    if (world < 1 || world > 1024) return NULL;
    trpo_hgroup *g = (trpo_hgroup *)calloc(1, sizeof(trpo_hgroup));
    if (!g) return NULL;
    g->world = world;
    g->slot = (double **)calloc(world, sizeof(double *));
    g->count = (size_t *)calloc(world, sizeof(size_t));
    g->attached = (int *)calloc(world, sizeof(int));
    if (!g->slot || !g->count || !g->attached || pthread_barrier_init(&g->bar, NULL, (unsigned)world) ||
        pthread_mutex_init(&g->mu, NULL)) {
        free(g->slot);
        free(g->count);
        free(g->attached);
        free(g);
        return NULL;
    }
    return g;
}

extern "C" void trpo_hgroup_destroy(trpo_hgroup *g) {
    if (!g) return;
    pthread_barrier_destroy(&g->bar);
    pthread_mutex_destroy(&g->mu);
    free(g->slot);
    free(g->count);
    free(g->attached);
    free(g);
}

// in-place sum of buf[count] (device, on d's stream) over the group; every rank must call it with
// the same count, in the same order as the others (the library's fixed launch sequences do)
__global__ void vcopy64_kernel(const double *__restrict__ src, double *__restrict__ dst, int n);
static int hgroup_allreduce(trpo_dev *d, double *buf, size_t count) {
    trpo_hgroup *g = d->group;
    // a local failure before the exchange still takes part in both barriers (a rank that returned
    // early would leave the others waiting forever): it publishes count (size_t)-1, which every rank
    // reads as a mismatch, so all of them return -4 together
    bool ok = true;
    if (count > d->gbuf_cap) {
        if (d->gbuf) hipHostFree(d->gbuf);
        d->gbuf = NULL;
        d->gbuf_cap = 0;
        ok = hipHostMalloc((void **)&d->gbuf, sizeof(double) * count, TRPO_HOST_COHERENT) == hipSuccess &&
             hipHostGetDevicePointer((void **)&d->gbuf_dev, d->gbuf, 0) == hipSuccess;
        if (ok) d->gbuf_cap = count;
    }
    // copies by KERNEL through the mapped buffer, not hipMemcpyAsync: a host-to-device hipMemcpyAsync
    // into buf followed by kernels reading buf gave intermittently stale reads (ranks diverging in
    // whole 512-element cg_axpy slices, 6 of 10 sharded 2x64 solves; tools/diag/shard_race.py)
    if (ok) hipLaunchKernelGGL(vcopy64_kernel, dim3(cdiv((long)count, 256)), dim3(256), 0, d->stream,
                               (const double *)buf, d->gbuf_dev, (int)count);
    ok = ok && hipGetLastError() == hipSuccess;
    ok = ok && hipStreamSynchronize(d->stream) == hipSuccess;
    g->slot[d->rank] = ok ? d->gbuf : NULL;
    g->count[d->rank] = ok ? count : (size_t)-1;
    pthread_barrier_wait(&g->bar);                 // every rank's partial (or failure) is published
    int bad = 0;
    for (int r = 0; r < g->world; ++r) bad |= g->count[r] != count;
    double *sum = bad ? NULL : (double *)malloc(sizeof(double) * (count ? count : 1));
    if (sum) {
        for (size_t i = 0; i < count; ++i) {
            double s = g->slot[0][i];
            for (int r = 1; r < g->world; ++r) s += g->slot[r][i];   // rank order: identical bits everywhere
            sum[i] = s;
        }
    }
    pthread_barrier_wait(&g->bar);                 // every rank has read every slot
    if (!sum) return -4;
    memcpy(d->gbuf, sum, sizeof(double) * count);
    free(sum);
    hipLaunchKernelGGL(vcopy64_kernel, dim3(cdiv((long)count, 256)), dim3(256), 0, d->stream,
                       (const double *)d->gbuf_dev, buf, (int)count);
    HCHK(hipGetLastError());
    DSYNC(d);
    return 0;
}

static int act_code(char a) {
    switch (a) {
    case 'l': return ACT_L;
    case 't': return ACT_T;
    case 'o': return ACT_O;
    case 's': return ACT_S;
    default: return -1;
    }
}



extern "C" size_t trpo_dev_num_params(const trpo_dev *d) { return d ? (size_t)d->P : 0; }

static void name_fast(trpo_dev *d) {
    const int *T = d->fast->T;
    const int no = d->coop ? 0 : d->fast->no;
    snprintf(d->name, sizeof d->name, "mfma-mlp3 %dx%dx%dx%d%s%s%s%s", T[0], T[1], T[2], T[3],
             d->fast->act >= 0 ? " ttl" : "", d->coop ? (d->coop_e->no ? " no4 coop" : " coop") : "",
             d->f64 ? " fp64" : "", !no ? "" : (no & NO_MFMA_RGW2) ? " no-mfma" : " no-valu");
}

// the narrow-output twin for n local samples: RGW2 on the VALU once every wave runs several tiles
// (its 16-column epilogue reduction then amortises; measured crossover between 50k and 500k samples on
// 256 blocks of 8 waves, TRPO_NO_VALU_MIN_TILES), else on the 16x16x4 contraction
static void bind_fast_no(trpo_dev *d) {
    if (!d->fast_no[0]) return;
    const char *e = getenv("TRPO_NO_VALU_MIN_TILES");
    const long min_tiles = e ? atol(e) : 4;
    const long tiles_per_wave = cdiv(cdiv((long)d->n, 16), (long)d->grid * d->fast_no[0]->waves);
    const FastEntry *f = d->fast_no[tiles_per_wave >= min_tiles ? 1 : 0];
    if (f == d->fast) return;
    d->fast = f;
    d->k_fvp = f->launch;
    d->k_pg = f->launch_pg;
    d->k_fvp_yc = f->launch_yc;
    d->k_cg_yc = f->launch_yc_cg[0];
    for (int i = 0; i < 4; ++i) d->k_cg_yc_q[i] = f->launch_yc_cg[i];
    d->yc_valid = 0;                                   // the two twins lay the y3 cache out alike, but be safe
    name_fast(d);
}

// force_prec: -1 = TRPO_PRECISION from the environment, 0 fp32, 1 fp64 (trpo_dev_create_prec: the
// fp64 twin of a context, built while other threads may create ordinary contexts)
static trpo_dev *dev_create(int device, size_t nl, const size_t *ls, const char *ac, int force_prec, char *err,
                            size_t errlen);
extern "C" trpo_dev *trpo_dev_create_prec(int device, size_t nl, const size_t *ls, const char *ac, int f64,
                                          char *err, size_t errlen) {
    return dev_create(device, nl, ls, ac, f64 ? 1 : 0, err, errlen);
}
extern "C" trpo_dev *trpo_dev_create(int device, size_t nl, const size_t *ls, const char *ac, char *err,
                                     size_t errlen) {
    return dev_create(device, nl, ls, ac, -1, err, errlen);
}
static trpo_dev *dev_create(int device, size_t nl, const size_t *ls, const char *ac, int force_prec, char *err,
                            size_t errlen) {
#define FAIL(...)                                      \
    do {                                               \
        if (err) snprintf(err, errlen, __VA_ARGS__);   \
        trpo_dev_destroy(d);                           \
        return NULL;                                   \
    } while (0)
    trpo_dev *d = NULL;
    if (nl < 2 || nl > MAXL || !ls || !ac) {
        if (err) snprintf(err, errlen, "invalid network description (NumLayers=%zu)", nl);
        return NULL;
    }
    d = (trpo_dev *)calloc(1, sizeof(trpo_dev));
    if (!d) return NULL;
    d->comm = NULL;
    d->world = 1;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) FAIL("no HIP device available");
    if (device < 0) {
        const char *e = getenv("TRPO_DEVICE");
        device = e ? atoi(e) : 0;
    }
    if (device >= ndev) FAIL("device %d out of range (%d devices)", device, ndev);
    d->device = device;
    if (hipSetDevice(device) != hipSuccess) FAIL("hipSetDevice(%d) failed", device);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        FAIL("device %d is %s; this library is built for gfx950 (MI355X) only", device, prop.gcnArchName);
    Net &n = d->net;
    memset(&n, 0, sizeof n);
    n.nl = (int)nl;
    int pos = 0;
    for (size_t i = 0; i < nl; ++i) {
        if (ls[i] == 0 || ls[i] > 65536) FAIL("LayerSize[%zu]=%zu unsupported", i, ls[i]);
        n.L[i] = (int)ls[i];
        if (i > 0) {
            n.act[i] = act_code(ac[i]);
            if (n.act[i] < 0) FAIL("AC Function for Layer[%zu] is %c. Unsupported.", i, ac[i]);
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
    d->P = n.P;
    d->Ps = (n.P + 1) & ~1;
    d->nw = n.P - n.A;
    if (d->P > 32 * 1024) FAIL("NumParams=%d exceeds the 32768 supported by the device CG", d->P);

    // pick the kernel family
    d->fast = d->fast_no[0] = d->fast_no[1] = NULL;
    if (nl == 4) {
        int T[4];
        for (int i = 0; i < 4; ++i) T[i] = cdiv(n.L[i], 16);
        const FastEntry *best = NULL;
        const int act = n.act[1] | (n.act[2] << 2) | (n.act[3] << 4);
        for (const FastEntry &f : kFast) {
            bool ok = (f.act < 0 || f.act == act) && f.no == 0;
            for (int i = 0; i < 4; ++i) ok = ok && f.T[i] >= T[i];
            if (!ok) continue;
            int cost = f.T[0] * f.T[1] + f.T[1] * f.T[2] + f.T[2] * f.T[3];
            int bcost = best ? best->T[0] * best->T[1] + best->T[1] * best->T[2] + best->T[2] * best->T[3] : 1 << 30;
            if (cost < bcost || (cost == bcost && best && best->act < 0 && f.act >= 0)) best = &f;
        }
        d->fast = best;
        // the narrow output layer's twins of that kernel (TRPO_NARROW_OUT, default on) where the
        // outputs fit: <= 3 -> the 3-output kernels, 4 -> the 4-output ones; set_obs picks one by N
        const char *eno = getenv("TRPO_NARROW_OUT");
        const int want = (!best || (eno && atoi(eno) == 0)) ? 0 : n.L[3] <= 3 ? 3 : n.L[3] <= 4 ? 4 : 0;
        d->fast_no[0] = d->fast_no[1] = NULL;
        if (want)
            for (const FastEntry &f : kFast) {
                bool same = f.act == best->act;
                for (int i = 0; i < 4; ++i) same = same && f.T[i] == best->T[i];
                if (same && f.no == (want | NO_MFMA_RGW2)) d->fast_no[0] = &f;
                if (same && f.no == want) d->fast_no[1] = &f;
            }
        if (!d->fast_no[0] || !d->fast_no[1]) d->fast_no[0] = d->fast_no[1] = NULL;
        if (d->fast_no[0]) d->fast = d->fast_no[0];
    }
    const char *force = getenv("TRPO_FORCE_GENERIC");
    if (force && atoi(force)) d->fast = d->fast_no[0] = d->fast_no[1] = NULL;
    {
        // precision mode: "fp64" runs the FVP in fp64 (v_mfma_f64_16x16x4_f64) -- the reference's
        // own precision -- through the cooperative kernel, which covers every tile-kernel shape
        const char *ep = force_prec >= 0 ? (force_prec ? "fp64" : "fp32") : getenv("TRPO_PRECISION");
        d->f64 = ep && (strcmp(ep, "fp64") == 0 || strcmp(ep, "64") == 0 || strcmp(ep, "double") == 0);
        if (ep && !d->f64 && strcmp(ep, "fp32") != 0 && strcmp(ep, "32") != 0 && strcmp(ep, "float") != 0)
            FAIL("TRPO_PRECISION=%s: expected fp32 or fp64", ep);
        d->esz = d->f64 ? sizeof(double) : sizeof(float);
    }

    if (hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess) FAIL("stream create failed");
    if (hipHostMalloc((void **)&d->wflag, 64, TRPO_HOST_COHERENT) == hipSuccess) {
        memset(d->wflag, 0, 64);
        if (hipHostGetDevicePointer((void **)&d->wflag_dev, d->wflag, 0) != hipSuccess) d->wflag_dev = NULL;
    } else {
        d->wflag = NULL;                          // trpo_dev_wait_done then synchronises the stream
    }
    if (hipEventCreate(&d->ev0) != hipSuccess || hipEventCreate(&d->ev1) != hipSuccess) FAIL("event create");
    d->hist_cap = 0;
#define DMALLOC(p, bytes)                                                   \
    do {                                                                    \
        if (trpo_malloc((void **)&(p), (bytes)) != hipSuccess) FAIL("trpo_malloc(%zu) failed", (size_t)(bytes)); \
        hipMemsetAsync((p), 0, (bytes), d->stream);                         \
    } while (0)
    DMALLOC(d->theta64, sizeof(double) * d->P);
    DMALLOC(d->std64, sizeof(double) * n.A);
    for (int i = 0; i < 5; ++i) DMALLOC(d->vec[i], sizeof(double) * d->Ps);
    DMALLOC(d->r, sizeof(double) * d->Ps);
    DMALLOC(d->zacc, sizeof(double) * d->Ps);
    DMALLOC(d->ctl, sizeof(Ctl));
    DMALLOC(d->st, 2 * sizeof(CgSt));
    for (int i = 0; i < 2; ++i) {
        DMALLOC(d->pbuf[i], sizeof(double) * d->Ps);
        DMALLOC(d->rbuf[i], sizeof(double) * d->Ps);
    }
    {
        const char *er = getenv("TRPO_REPLICAS");
        d->R = er ? atoi(er) : RMAX;
        if (d->R < 1) d->R = 1;
        if (d->R > RMAX) d->R = RMAX;
    }
    DMALLOC(d->accbuf, sizeof(double) * 3 * d->R * d->Ps);
    DMALLOC(d->qbuf, sizeof(double) * QCAP * d->Ps);
    DMALLOC(d->qzero, sizeof(double) * 64);
    {
        const char *el = getenv("TRPO_CG_LAST");
        d->no_cg_last = el && atoi(el) == 0;
        // residual reorthogonalisation counters the fp32 FVP's direction-dependent noise; the
        // fp64 mode has none to counter and runs the reference's plain CG: where the reference's own
        // fp64 CG loses orthogonality (random-shape draw 23: a stalled solve), reorthogonalising would
        // move the step 1.2e-3 AWAY from the reference (1.0e-5 without; tools/diag/draw23.py)
        const char *eo = getenv("TRPO_CG_REORTH");
        d->reorth = eo ? atoi(eo) != 0 : !d->f64;
    }
    DMALLOC(d->pacc, sizeof(double) * 2 * d->R * d->Ps);
    d->Rc = d->R;
    if (d->fast) {
        Pack &pk = d->pack;
        for (int i = 0; i < 4; ++i) pk.T[i] = d->fast->T[i];
        const int *T = pk.T;
        pk.fa[0] = 0;
        pk.fa[1] = pk.fa[0] + 256 * T[0] * T[1];
        pk.fa[2] = pk.fa[1] + 256 * T[1] * T[2];
        pk.fb[0] = -1;
        pk.fb[1] = pk.fa[2] + 256 * T[2] * T[3];
        pk.fb[2] = pk.fb[1] + 256 * T[1] * T[2];
        pk.bi[0] = pk.fb[2] + 256 * T[2] * T[3];
        pk.bi[1] = pk.bi[0] + 16 * T[1];
        pk.bi[2] = pk.bi[1] + 16 * T[2];
        pk.iv = pk.bi[2] + 16 * T[3];
        pk.tlen = pk.iv + 16 * T[3];
        pk.vfa[0] = 0;
        pk.vfa[1] = pk.vfa[0] + 256 * T[0] * T[1];
        pk.vfa[2] = pk.vfa[1] + 256 * T[1] * T[2];
        pk.vb[0] = pk.vfa[2] + 256 * T[2] * T[3];
        pk.vb[1] = pk.vb[0] + 16 * T[1];
        pk.vb[2] = pk.vb[1] + 16 * T[2];
        pk.vlen = pk.vb[2] + 16 * T[3];
        if (pk.tlen != d->fast->tlen || pk.vlen != d->fast->vlen) FAIL("internal: pack layout mismatch");
        if (pk.vlen > VPACK_PER_THREAD * 1024) FAIL("internal: direction pack of %d exceeds the CG kernels' %d",
                                                    pk.vlen, VPACK_PER_THREAD * 1024);
        DMALLOC(d->tpack, d->esz * pk.tlen);
        DMALLOC(d->vpack, d->esz * pk.vlen);
        DMALLOC(d->tmap, sizeof(int) * pk.tlen);
        DMALLOC(d->vmap, sizeof(int) * pk.vlen);
        DMALLOC(d->pslot, sizeof(int) * d->Ps);
        hipLaunchKernelGGL(build_pslot_kernel, dim3(cdiv(d->P, 256)), dim3(256), 0, d->stream, n, pk, d->pslot, d->P);
        DMALLOC(d->islot, sizeof(int) * (d->nw > 0 ? d->nw : 1));
        hipLaunchKernelGGL(build_islot_kernel, dim3(cdiv(d->nw, 256)), dim3(256), 0, d->stream, n, pk, d->islot, d->nw);
        const int len = pk.tlen > pk.vlen ? pk.tlen : pk.vlen;
        hipLaunchKernelGGL(build_maps_kernel, dim3(cdiv(len, 256)), dim3(256), 0, d->stream, n, pk, d->tmap, d->vmap,
                           d->f64);
        if (d->fast->attr(d->fast->lds) != hipSuccess) FAIL("hipFuncSetAttribute(LDS=%d) failed", d->fast->lds);
        if (d->fast_no[1] && d->fast_no[1]->attr(d->fast_no[1]->lds) != hipSuccess)
            FAIL("hipFuncSetAttribute(LDS=%d) failed", d->fast_no[1]->lds);
        d->k_fvp = d->fast->launch;
        d->k_pg = d->fast->launch_pg;
        d->k_lds = d->fast->lds;
        d->k_tiles = d->fast->waves;
        d->slab = d->fast->slab;
        // wide hidden layers: the cooperative kernel (TRPO_COOP=0 keeps the one-wave-per-tile kernel)
        d->coop_e = NULL;
        d->coop = 0;
        const char *ec = getenv("TRPO_COOP");
        const char *eno_coop = getenv("TRPO_NARROW_OUT");
        if ((d->f64 || !(ec && atoi(ec) == 0)) && T[1] == T[2] && T[3] == 1)
            for (const CoopEntry &e : kCoop)
                if (e.f64 == d->f64 && e.T0 == T[0] && e.TH == T[1] && e.act == d->fast->act && e.no == 0)
                    d->coop_e = &e;
        // its narrow-output twin (fp32, <= 4 outputs; TRPO_NARROW_OUT=0 keeps the 16x16x4 output layer)
        if (d->coop_e && !d->f64 && n.L[3] <= 4 && !(eno_coop && atoi(eno_coop) == 0))
            for (const CoopEntry &e : kCoop)
                if (!e.f64 && e.T0 == T[0] && e.TH == T[1] && e.act == d->fast->act && e.no == 4) d->coop_e = &e;
        if (d->f64 && !d->coop_e) FAIL("internal: no fp64 kernel for tile shape %dx%dx%dx%d", T[0], T[1], T[2], T[3]);
        if (d->coop_e) {
            if (d->coop_e->attr(d->coop_e->lds) != hipSuccess)
                FAIL("hipFuncSetAttribute(LDS=%d) failed", d->coop_e->lds);
            d->coop = 1;
            d->k_fvp = d->coop_e->launch;
            d->k_pg = d->coop_e->launch_pg;
            d->k_lds = d->coop_e->lds;
            d->k_tiles = d->coop_e->ng;
            d->slab = d->coop_e->slab;
            const char *ef = getenv("TRPO_COOP_FUSED");
            d->coop_fused = !(ef && atoi(ef) == 0) &&
                            (size_t)d->coop_e->main_bytes >=
                                sizeof(double) * (d->P + 2 + 128 + QCAP * 4 * (d->coop_e->threads / 64));
            // the distributed step forms |r'|^2 from the dots (|r|^2 - 2a r.z + a^2 z.z - sum c^2), as
            // the fused small-net step does: in fp32 the FVP noise floor keeps |r'|^2 / |r|^2 far above
            // fp64 rounding, but an fp64 solve that converges to ~1e-14 and keeps iterating (ResidualTh 0)
            // cancels that difference to noise (measured: [32,16,16,1] 'lotl' fp64 9e-2 off), so the fp64
            // mode keeps the fused cooperative step with its direct |r'|^2 reduction
            const char *ed = getenv("TRPO_COOP_DIST");
            d->coop_dist = !d->f64 && !(ed && atoi(ed) == 0);
            // the FVP after each distributed step loads p' from the fragment-order pack cg_axpy scattered it
            // into (coalesced) instead of gathering it element by element in every block's prologue
            const char *epk = getenv("TRPO_COOP_PK");
            d->coop_pk = d->coop_dist && !(epk && atoi(epk) == 0);
            const char *eci = getenv("TRPO_COOP_CINIT");
            d->cinit = !(eci && atoi(eci) == 0);         // (read for both cooperative CG forms)
            DMALLOC(d->zbuf, sizeof(double) * d->Ps);
            const char *egm = getenv("TRPO_COOP_GMAJ");
            d->coop_gmaj = egm ? (atoi(egm) != 0) : -1;
            const char *erd = getenv("TRPO_COOP_RDOTS");
            d->coop_rdots = d->coop_dist && !(erd && atoi(erd) == 0) && d->P - d->nw <= RS_THREADS - RS_POS;
            {
                const int gd = cdiv(d->Ps / 2, CGS_T), gr = d->slab / RS_POS;   // cg_dots / reduce_dots partials
                DMALLOC(d->dotsbuf, sizeof(double) * CGS_K * (gd > gr ? gd : gr));
            }
            DMALLOC(d->imap, sizeof(int) * d->slab);
            hipLaunchKernelGGL(build_imap_coop_kernel, dim3(cdiv(d->slab, 256)), dim3(256), 0, d->stream, n, T[0],
                               T[1], d->f64, d->coop_e->no, d->imap, d->slab);
        } else {
            DMALLOC(d->imap, sizeof(int) * d->slab);
            hipLaunchKernelGGL(build_imap_kernel, dim3(cdiv(d->slab, 256)), dim3(256), 0, d->stream, n, pk, d->imap,
                               d->slab);
        }
        {
            // forward cache: small-net one-wave kernel (MODE 2/3), or the fp32 cooperative kernel
            // (MODE 3/4) when the output activation needs no y (its y3 is not cached)
            const char *ey = getenv("TRPO_YCACHE");
            if (d->coop) {
                d->k_fvp_yc = d->coop_e->launch_yc;
                d->k_cg_yc = d->coop_e->launch_cg_yc;
                if (n.act[3] == ACT_T || n.act[3] == ACT_S) d->k_fvp_yc = d->k_cg_yc = NULL;
            } else {
                d->k_fvp_yc = d->fast->launch_yc;
                d->k_cg_yc = d->fast->launch_yc_cg[0];
                for (int i = 0; i < 4; ++i) d->k_cg_yc_q[i] = d->fast->launch_yc_cg[i];
            }
            d->yc_on = d->k_fvp_yc && d->k_cg_yc && !(ey && atoi(ey) == 0);
        }
        if (d->coop) d->fast_no[0] = d->fast_no[1] = NULL;
        name_fast(d);
    } else {
        d->esz = d->f64 ? sizeof(double) : sizeof(float);
        DMALLOC(d->gth, d->esz * d->P);
        DMALLOC(d->gv, d->esz * d->P);
        DMALLOC(d->giv, d->esz * n.A);
        int rows = 0;
        for (int i = 0; i < n.nl; ++i) rows += n.L[i];
        d->srows = rows;
        d->slab = cdiv(d->P, RS_POS) * RS_POS;           // row stride of the block partials
        DMALLOC(d->imap, sizeof(int) * d->slab);
        hipLaunchKernelGGL(iota_kernel, dim3(cdiv(d->slab, 256)), dim3(256), 0, d->stream, d->imap, d->slab, d->nw);
        snprintf(d->name, sizeof d->name, "generic%s", d->f64 ? " fp64" : "");
    }
    if (hipStreamSynchronize(d->stream) != hipSuccess) FAIL("initialisation kernels failed");
    d->damping = 0.1;
    d->n_total = 0;
    Ctl c0;
    memset(&c0, 0, sizeof c0);
    c0.damping = d->damping;
    if (hipMemcpyAsync(d->ctl, &c0, sizeof c0, hipMemcpyHostToDevice, d->stream) != hipSuccess ||
        hipStreamSynchronize(d->stream) != hipSuccess)
        FAIL("control block upload failed");
    return d;
#undef FAIL
#undef DMALLOC
}

// Diagnostics (TRPO_DEBUG_ALLOC=1, stderr): the device address range of every buffer of the context, so
// a probe can see whether a context's buffers reuse pages of an earlier context's freed peer window
// (the peer-path wrong results under torch's runtime).
static void dbg_dump(trpo_dev *d, const char *tag) {
    if (!getenv("TRPO_DEBUG_ALLOC")) return;
    const void *ptrs[] = {d->zbuf, d->dotsbuf, d->obs64, d->pg_d, d->pg_adv, d->pg_iv, d->st, d->pbuf[0], d->pbuf[1], d->rbuf[0], d->rbuf[1], d->accbuf, d->pacc, d->imap, d->tpack, d->vpack, d->tmap, d->vmap, d->pslot, d->islot, d->obs4, d->yc, d->gth, d->gv, d->giv, d->gobs, d->scratch,
                          d->theta64, d->std64, d->r, d->zacc, d->slabs, d->ctl, d->hist, d->tscr, d->qbuf, d->qzero, d->zred, d->ptmp, d->pn, d->vec[0], d->vec[1], d->vec[2], d->vec[3], d->vec[4]};
    const char *names[] = {"zbuf", "dotsbuf", "obs64", "pg_d", "pg_adv", "pg_iv", "st", "pbuf0", "pbuf1", "rbuf0", "rbuf1", "accbuf", "pacc", "imap", "tpack", "vpack", "tmap", "vmap", "pslot", "islot", "obs4", "yc", "gth", "gv", "giv", "gobs", "scratch",
                           "theta64", "std64", "r", "zacc", "slabs", "ctl", "hist", "tscr", "qbuf", "qzero", "zred", "ptmp", "pn", "vec0", "vec1", "vec2", "vec3", "vec4"};
    static_assert(sizeof(ptrs) / sizeof(ptrs[0]) == sizeof(names) / sizeof(names[0]), "names");
    for (size_t i = 0; i < sizeof(ptrs) / sizeof(ptrs[0]); ++i) {
        if (!ptrs[i]) continue;
        void *base = NULL;
        size_t sz = 0;
        if (hipMemPtrGetInfo((void *)ptrs[i], &sz) != hipSuccess) (void)hipGetLastError();
        base = (void *)ptrs[i];
        fprintf(stderr, "[trpo_alloc] %s ctx=%p %s %p +%zu\n", tag, (void *)d, names[i], base, sz);
    }
    if (d->peer) fprintf(stderr, "[trpo_alloc] %s ctx=%p window %p\n", tag, (void *)d, trpo_peer_window(d->peer));
}

extern "C" void trpo_dev_destroy(trpo_dev *d) {
    if (!d) return;
    dbg_dump(d, "destroy");
    if (d->stream) hipStreamSynchronize(d->stream);
    if (d->cg_exec) hipGraphExecDestroy(d->cg_exec);
    if (d->comm) ncclCommDestroy(d->comm);
    trpo_peer_destroy(d->peer);
    trpo_update_state_free(d->upd);
    void *ptrs[] = {d->zbuf, d->dotsbuf, d->obs64, d->pg_d, d->pg_adv, d->pg_iv, d->st, d->pbuf[0], d->pbuf[1], d->rbuf[0], d->rbuf[1], d->accbuf, d->pacc, d->imap, d->tpack, d->vpack, d->tmap, d->vmap, d->pslot, d->islot, d->obs4, d->yc, d->gth, d->gv, d->giv, d->gobs, d->scratch,
                    d->theta64, d->std64, d->r, d->zacc, d->slabs, d->ctl, d->hist, d->tscr, d->qbuf, d->qzero, d->zred, d->ptmp, d->pn};
    for (void *p : ptrs)
        if (p) hipFree(p);
    for (int i = 0; i < 5; ++i)
        if (d->vec[i]) hipFree(d->vec[i]);
    if (d->hst) hipHostFree(d->hst);
    if (d->gbuf) hipHostFree(d->gbuf);
    if (d->wflag) hipHostFree(d->wflag);
    if (d->ev0) hipEventDestroy(d->ev0);
    if (d->ev1) hipEventDestroy(d->ev1);
    if (d->stream) hipStreamDestroy(d->stream);
    free(d);
}

static int sync_ctl_scalars(trpo_dev *d) {
    // damping and N live in the control block so captured graphs stay valid
    HCHK(hipMemcpyAsync(&d->ctl->damping, &d->damping, sizeof(double), hipMemcpyHostToDevice, d->stream));
    HCHK(hipMemcpyAsync(&d->ctl->n_total, &d->n_total, sizeof(double), hipMemcpyHostToDevice, d->stream));
    DSYNC(d);
    return 0;
}

extern "C" int trpo_dev_set_damping(trpo_dev *d, double damping) {
    if (!d) return -1;
    HCHK(hipSetDevice(d->device));
    d->damping = damping;
    return sync_ctl_scalars(d);
}

extern "C" int trpo_dev_set_theta(trpo_dev *d, const double *theta) {
    if (!d || !theta) return -1;
    HCHK(hipSetDevice(d->device));
    HCHK(hipMemcpyAsync(d->theta64, theta, sizeof(double) * d->P, hipMemcpyHostToDevice, d->stream));
    d->yc_valid = 0;
    if (d->fast) {
        hipLaunchKernelGGL(gather_pack_kernel, dim3(cdiv(d->pack.iv, 256)), dim3(256), 0, d->stream, d->tpack,
                           d->theta64, d->tmap, d->pack.iv, d->f64);
    } else {
        hipLaunchKernelGGL(to_elem_kernel, dim3(cdiv(d->P, 256)), dim3(256), 0, d->stream, d->gth, d->theta64,
                           (long)d->P, d->f64);
    }
    HCHK(hipGetLastError());
    DSYNC(d);
    return 0;
}

extern "C" int trpo_dev_set_std(trpo_dev *d, const double *stdv) {
    if (!d || !stdv) return -1;
    HCHK(hipSetDevice(d->device));
    for (int j = 0; j < d->net.A; ++j)
        if (!(stdv[j] > 0.0) && !(stdv[j] < 0.0)) return -1;     // sigma must be non-zero
    HCHK(hipMemcpyAsync(d->std64, stdv, sizeof(double) * d->net.A, hipMemcpyHostToDevice, d->stream));
    if (d->fast) {
        const int len = 16 * d->pack.T[3];
        hipLaunchKernelGGL(set_invvar_kernel, dim3(1), dim3(cdiv(len, 64) * 64), 0, d->stream,
                           (void *)((char *)d->tpack + d->esz * d->pack.iv), d->std64, d->net.A, len, d->f64);
    } else {
        hipLaunchKernelGGL(set_invvar_kernel, dim3(cdiv(d->net.A, 256)), dim3(256), 0, d->stream, d->giv,
                           d->std64, d->net.A, d->net.A, d->f64);
    }
    HCHK(hipGetLastError());
    DSYNC(d);
    return 0;
}

static void choose_reduction(trpo_dev *d) {
    // fused single-kernel CG iterations with fp64 atomics when the block partials are small
    // (G x P values per FVP); otherwise block slabs + a reduce kernel
    // decided from P only, so every rank of a sharded run picks the same collective pattern
    const char *e = getenv("TRPO_ATOMIC");
    const bool ok = d->fast && !d->coop && !d->f64 && d->fast->emax <= 4 && d->P <= 2048;
    d->atomic = ok && 256L * d->P <= 400000;
    if (e) d->atomic = ok && atoi(e) != 0;
}

static int choose_grid(trpo_dev *d) {
    // one 8-wave block per CU at most; at least one tile per wave
    int cus = 256;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, d->device) == hipSuccess && prop.multiProcessorCount > 0)
        cus = prop.multiProcessorCount;
    const char *e = getenv("TRPO_FVP_BLOCKS");
    if (d->fast) {
        const int ntiles = cdiv((long)d->n, 16);
        // cooperative kernel, group-major tiles (A.gmaj): by default when the grid is full either way
        // (ntiles >= groups of a full grid), and at <= cus / 2 tiles.  In between group-major spreads the
        // busy groups one per block over up to twice the blocks and the slab reduce reads twice the block
        // partials: 2x64 N = 4 096 (256 tiles) kernel 8.44 -> 7.73 us but FVP call 11.75 -> 12.18 us and CG
        // 197.0 -> 202.0 us, while at N = 2 048 (128 tiles) kernel 8.31 -> 7.16 us, call 11.21 -> 10.59 us,
        // CG 192.0 -> 185.8 us (profiles/r05_ab_coop.log); TRPO_COOP_GMAJ=1 / 0 forces it on / off
        d->gmaj_on = d->coop && (d->coop_gmaj > 0 ||
                                 (d->coop_gmaj < 0 && (ntiles >= d->k_tiles * cus || 2 * ntiles <= cus)));
        // a standalone FVP call (slab reduce + epilogue, no CG dots) takes group-major tiles up to one tile
        // per CU as well, while the CG launches keep the rule above (at N = 4 096 the CG is faster
        // block-major: 192.8 vs 198.2 us).  2x64 FVP kernel at N = 3 000 (188 tiles) 7.89 -> 7.05 and
        // 8.65 -> 8.18 us; at N = 4 096 (256 tiles, every CU one block) 7.93 -> 7.43, 8.02 -> 8.15 and
        // 8.16 -> 8.18 us in three runs; at 6 144 it loses (profiles/r05_gmaj_fvp_ab.log).  fp32 only.
        d->gmaj_fvp = d->gmaj_on || (d->coop && !d->f64 && d->coop_gmaj < 0 && ntiles <= cus);
        auto grid_of = [&](int gm) {
            int g = cdiv(ntiles, gm ? 1 : d->k_tiles);
            if (g > cus) g = cus;
            if (e && atoi(e) > 0) g = atoi(e);
            return g < 1 ? 1 : g;
        };
        d->grid_fvp = grid_of(d->gmaj_fvp);
        return grid_of(d->gmaj_on);
    }
    const int npass = cdiv((long)d->n, GEN_T);
    int g = npass < cus ? npass : cus;
    if (e && atoi(e) > 0) g = atoi(e);
    d->gmaj_fvp = 0;
    d->grid_fvp = g < 1 ? 1 : g;
    return g < 1 ? 1 : g;
}

static int refresh_n_total(trpo_dev *d);
static int allreduce(trpo_dev *d, double *buf, size_t count);

extern "C" int trpo_dev_set_obs(trpo_dev *d, const double *obs, size_t n) {
    if (!d || (!obs && n) || n > (size_t)1 << 30) return -1;
    HCHK(hipSetDevice(d->device));
    const int L0 = d->net.L[0];
    double *tmp = NULL;
    if (n) {
        HCHK(trpo_malloc((void **)&tmp, sizeof(double) * n * L0));
        HCHK(hipMemcpyAsync(tmp, obs, sizeof(double) * n * L0, hipMemcpyHostToDevice, d->stream));
    }
    d->n = n;
    d->grid = choose_grid(d);
    choose_reduction(d);
    bind_fast_no(d);
    if (d->fast) {
        const size_t npad = (size_t)cdiv((long)n, 16) * 16 + 16;
        const int ld = 16 * d->pack.T[0];
        if (npad > d->npad_cap) {
            if (d->obs4) hipFree(d->obs4);
            HCHK(trpo_malloc((void **)&d->obs4, d->esz * npad * ld));
            d->npad_cap = npad;
        }
        if (n)
            hipLaunchKernelGGL(obs_pad_kernel, dim3(cdiv((long)npad * ld, 256)), dim3(256), 0, d->stream,
                               d->obs4, tmp, (int)n, (int)npad, L0, ld, d->f64);
        d->yc_valid = 0;
        if (d->yc_on) {
            const int *T = d->pack.T;
            const size_t bytes = (size_t)(npad / 16) * (T[1] + T[2] + T[3]) * 64 * 4 * d->esz;
            if (bytes > d->yc_cap) {
                if (d->yc) hipFree(d->yc);
                d->yc = NULL;
                d->yc_cap = 0;
                HCHK(trpo_malloc(&d->yc, bytes));
                d->yc_cap = bytes;
            }
        }
    } else {
        if ((size_t)n * L0 > d->npad_cap) {
            if (d->gobs) hipFree(d->gobs);
            HCHK(trpo_malloc((void **)&d->gobs, d->esz * (n * L0 + 1)));
            d->npad_cap = n * L0;
        }
        if (n) hipLaunchKernelGGL(to_elem_kernel, dim3(cdiv((long)n * L0, 256)), dim3(256), 0, d->stream, d->gobs,
                                  tmp, (long)n * L0, d->f64);
        if ((size_t)d->grid > d->scratch_blocks) {
            if (d->scratch) hipFree(d->scratch);
            HCHK(trpo_malloc((void **)&d->scratch, d->esz * 3 * (size_t)d->srows * GEN_T * d->grid));
            d->scratch_blocks = d->grid;
        }
    }
    const int sblocks = d->grid > d->grid_fvp ? d->grid : d->grid_fvp;     // CG and FVP-call grids
    if (sblocks > d->slab_blocks) {
        if (d->slabs) hipFree(d->slabs);
        HCHK(trpo_malloc((void **)&d->slabs, d->esz * (size_t)d->slab * sblocks));
        HCHK(hipMemsetAsync(d->slabs, 0, d->esz * (size_t)d->slab * sblocks, d->stream));
        d->slab_blocks = sblocks;
    }
    HCHK(hipGetLastError());
    DSYNC(d);
    if (d->obs64) hipFree(d->obs64);
    d->obs64 = tmp;                                    // kept in fp64 for the TRPO_Update path
    if (d->cg_exec) {     // geometry may have changed: recapture next time
        hipGraphExecDestroy(d->cg_exec);
        d->cg_exec = NULL;
    }
    return refresh_n_total(d);
}

// Replicas of the atomic partial sums in use.  One GPU: R (8; 32 block adds per address at 256
// blocks measured best).  Under RCCL every rank all-reduces Rc x P values per FVP, so Rc is sized
// for ~32 adds per address from the LARGEST shard's grid -- computed from global quantities only,
// so it is identical on every rank (the collective's count must match).
static int choose_replicas(trpo_dev *d) {
    int rc = d->R;
    if (d->world > 1 && d->fast) {
        int cus = 256;
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, d->device) == hipSuccess && prop.multiProcessorCount > 0)
            cus = prop.multiProcessorCount;
        const long nmax = (long)d->n_max;                 // the largest shard over all ranks
        long g = cdiv(cdiv(nmax, 16), d->k_tiles);
        if (g > cus) g = cus;
        rc = (int)cdiv(g, 32);
    }
    const char *eu = getenv("TRPO_REPLICAS_USED");      // testing: force the multi-rank sizing on one GPU
    if (eu && atoi(eu) > 0) rc = atoi(eu);
    if (rc < 1) rc = 1;
    if (rc > d->R) rc = d->R;
    if (rc != d->Rc) {
        // a different prefix of each replica set is used from now on: start from all-zero sets
        HCHK(hipMemsetAsync(d->accbuf, 0, sizeof(double) * 3 * d->R * d->Ps, d->stream));
        HCHK(hipMemsetAsync(d->pacc, 0, sizeof(double) * 2 * d->R * d->Ps, d->stream));
        DSYNC(d);
        d->Rc = rc;
        if (d->cg_exec) {
            hipGraphExecDestroy(d->cg_exec);
            d->cg_exec = NULL;
        }
    }
    return 0;
}

// N is the global sample count: local n, or the all-reduced n under RCCL
static int refresh_n_total(trpo_dev *d) {
    const size_t n = d->n;
    if (has_collective(d)) {
        // every rank's shard size in one sum-all-reduce (rank r contributes n at slot r): N is the
        // total, and the replica sizing below reads the LARGEST shard -- both identical on all ranks
        const int W = d->world;
        double *hn = (double *)calloc(W, sizeof(double)), *dn = d->peer_on ? d->pn : NULL;
        if (!hn) return -3;
        hn[d->rank] = (double)n;
        // the peer exchange uses a buffer allocated with its window: no allocation (which may wait for
        // the whole device) while another context of this process already spins in its exchange
        if (!dn && trpo_malloc((void **)&dn, sizeof(double) * W) != hipSuccess) {
            free(hn);
            return -2;
        }
        int rc = hipMemcpyAsync(dn, hn, sizeof(double) * W, hipMemcpyHostToDevice, d->stream) ? -2 : 0;
        if (!rc) rc = allreduce(d, dn, (size_t)W);
        if (!rc && hipMemcpyAsync(hn, dn, sizeof(double) * W, hipMemcpyDeviceToHost, d->stream)) rc = -2;
        if (!rc && hipStreamSynchronize(d->stream)) rc = -2;
        if (dn != d->pn) hipFree(dn);
        if (!rc) {
            double tot = 0.0, mx = 0.0;
            for (int r = 0; r < W; ++r) {
                tot += hn[r];
                mx = hn[r] > mx ? hn[r] : mx;
            }
            d->n_total = tot;
            d->n_max = mx;
        }
        free(hn);
        if (rc) return rc;
    } else {
        d->n_total = (double)n;
        d->n_max = (double)n;
    }
    if (choose_replicas(d)) return -2;
    return sync_ctl_scalars(d);
}

extern "C" int trpo_dev_comm_unique_id(void *id128) {
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return -4;
    memcpy(id128, &id, sizeof(id) < 128 ? sizeof(id) : 128);
    return 0;
}

extern "C" int trpo_dev_set_group(trpo_dev *d, trpo_hgroup *g, int rank) {
    if (!d || !g || rank < 0 || rank >= g->world) return -1;
    HCHK(hipSetDevice(d->device));
    if (d->comm) {
        ncclCommDestroy(d->comm);
        d->comm = NULL;
    }
    pthread_mutex_lock(&g->mu);
    const int taken = g->attached[rank];
    g->attached[rank] = 1;
    pthread_mutex_unlock(&g->mu);
    if (taken) return -1;
    d->peer_on = 0;
    d->group = g;
    d->rank = rank;
    d->world = g->world;
    if (d->cg_exec) {               // the host exchange cannot live in a graph: CG runs eagerly
        hipGraphExecDestroy(d->cg_exec);
        d->cg_exec = NULL;
    }
    return refresh_n_total(d);
}

// ranks of the attached communicator as the collective library itself reports them (RCCL's
// ncclCommCount), the context's rank, and the atomic replica sets in use
extern "C" int trpo_dev_comm_info(const trpo_dev *d, int *rank, int *world, int *replicas) {
    if (!d) return -1;
    int w = d->world;
    if (d->comm) {
        int c = 0;
        if (ncclCommCount(d->comm, &c) != ncclSuccess) return -4;
        w = c;
    }
    if (rank) *rank = d->rank;
    if (world) *world = w;
    if (replicas) *replicas = d->atomic ? d->Rc : 0;
    return 0;
}

// Bounded RCCL initialisation.  ncclCommInitRank blocks until every rank of the unique id has joined;
// a rank that never arrives (crashed, or failed before the call) would hold the others forever.  The
// call therefore runs in a helper thread and the caller waits at most timeout_ms: on time-out the
// attach fails (-6) and the helper is abandoned -- if its init completes later, it aborts the
// communicator itself.  The communicator stays a BLOCKING one, so the data path (eager and
// graph-captured ncclAllReduce) is exactly that of an ordinary ncclCommInitRank.
extern "C" int trpo_dev_comm_error(const trpo_dev *d);
static int ensure_hst(trpo_dev *d, size_t count, bool host_writes);
__global__ void vcopy64_kernel(const double *__restrict__ src, double *__restrict__ dst, int n);

struct CommInitJob {
    pthread_mutex_t mu;
    int device, world, rank;
    ncclUniqueId id;
    ncclComm_t comm;
    ncclResult_t res;
    int done, abandoned;
};

static void *comm_init_thread(void *arg) {
    CommInitJob *j = (CommInitJob *)arg;
    ncclComm_t c = NULL;
    ncclResult_t r = hipSetDevice(j->device) == hipSuccess ? ncclCommInitRank(&c, j->world, j->id, j->rank)
                                                             : ncclUnhandledCudaError;
    pthread_mutex_lock(&j->mu);
    j->comm = c;
    j->res = r;
    j->done = 1;
    const int abandoned = j->abandoned;
    pthread_mutex_unlock(&j->mu);
    if (abandoned) {
        if (r == ncclSuccess && c) ncclCommAbort(c);
        pthread_mutex_destroy(&j->mu);
        free(j);
    }
    return NULL;
}

static double mono_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return 1e3 * (double)ts.tv_sec + 1e-6 * (double)ts.tv_nsec;
}

static long comm_timeout_ms(long given) {
    if (given > 0) return given;
    const char *e = getenv("TRPO_COMM_TIMEOUT_MS");
    return e && atol(e) > 0 ? atol(e) : 120000;
}

static int comm_init_bounded(trpo_dev *d, int rank, int world, const void *id128, long timeout_ms) {
    CommInitJob *j = (CommInitJob *)calloc(1, sizeof(CommInitJob));
    if (!j) return -3;
    pthread_mutex_init(&j->mu, NULL);
    j->device = d->device;
    j->world = world;
    j->rank = rank;
    memcpy(&j->id, id128, sizeof(j->id));
    pthread_t th;
    if (pthread_create(&th, NULL, comm_init_thread, j) != 0) {
        pthread_mutex_destroy(&j->mu);
        free(j);
        return -3;
    }
    pthread_detach(th);
    const double t_end = mono_ms() + (double)timeout_ms;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        const int done = j->done;
        if (!done && mono_ms() > t_end) j->abandoned = 1;       // the helper frees the job
        const int abandoned = j->abandoned;
        pthread_mutex_unlock(&j->mu);
        if (done) break;
        if (abandoned) {
            fprintf(stderr, "[trpo_mi355x] ncclCommInitRank(rank %d of %d, device %d): no completion within %ld ms\n",
                    rank, world, d->device, timeout_ms);
            return -6;
        }
        struct timespec ts = {0, 1000000};
        nanosleep(&ts, NULL);
    }
    const ncclResult_t nr = j->res;
    ncclComm_t c = j->comm;
    pthread_mutex_destroy(&j->mu);
    free(j);
    if (nr != ncclSuccess) {
        fprintf(stderr, "[trpo_mi355x] ncclCommInitRank(rank %d of %d, device %d): %s\n", rank, world, d->device,
                ncclGetErrorString(nr));
        return -4;
    }
    d->comm = c;
    return 0;
}

extern "C" int trpo_dev_set_comm(trpo_dev *d, int rank, int world, const void *id128, long timeout_ms) {
    if (!d || world < 1 || rank < 0 || rank >= world || (world > 1 && !id128)) return -1;
    HCHK(hipSetDevice(d->device));
    d->group = NULL;
    d->peer_on = 0;
    d->comm_aborted = 0;
    if (d->comm) {
        ncclCommDestroy(d->comm);
        d->comm = NULL;
    }
    if (world > 1) {
        const int rc = comm_init_bounded(d, rank, world, id128, comm_timeout_ms(timeout_ms));
        if (rc) return rc;
    }
    d->rank = rank;
    d->world = world;
    if (d->cg_exec) {
        hipGraphExecDestroy(d->cg_exec);
        d->cg_exec = NULL;
    }
    return refresh_n_total(d);
}

// Wait for everything enqueued on the context's stream, at most timeout_ms (<= 0: the default of
// TRPO_COMM_TIMEOUT_MS / 120 s): 0 when it completed (or the collective's error), -6 on time-out.
// spin: poll without sleeping for the first WAIT_SPIN_MS (a timed region's closing wait must not add a
// sleep quantum), then 50 us between polls, so a slow or hung collective does not hold a host core at
// 100 % for the whole bound; otherwise 50 us between polls from the start.
#define WAIT_SPIN_MS 250.0
static int wait_stream(trpo_dev *d, long timeout_ms, bool spin) {
    const double t0 = mono_ms();
    const double t_end = t0 + (double)comm_timeout_ms(timeout_ms);
    for (;;) {
        const hipError_t e = hipStreamQuery(d->stream);
        if (e == hipSuccess) return 0;
        if (e != hipErrorNotReady) {
            fprintf(stderr, "[trpo_mi355x] HIP error %s while waiting for the stream\n", hipGetErrorString(e));
            return -2;
        }
        const double now = mono_ms();
        if (now > t_end) return -6;
        if (!spin || now - t0 > WAIT_SPIN_MS) {
            struct timespec ts = {0, 50000};
            nanosleep(&ts, NULL);
        }
    }
}

// The host's wait at the end of a synchronous call (update, FVP, surrogate, ...): a plain stream
// synchronisation on one rank; with a collective attached a peer that never arrives must not hang the
// caller, so the wait is bounded (TRPO_COMM_TIMEOUT_MS / 120 s) and reports -6 / the collective's error.
int trpo_dev_has_collective(const trpo_dev *d) { return has_collective(d) ? 1 : 0; }

extern "C" int trpo_dev_wait_done(trpo_dev *d) {
    if (!has_collective(d)) return hipStreamSynchronize(d->stream) == hipSuccess ? 0 : -2;
    const int rc = wait_stream(d, 0, true);
    return rc ? rc : trpo_dev_comm_error(d);
}

extern "C" int trpo_dev_wait(trpo_dev *d, long timeout_ms) {
    if (!d) return -1;
    HCHK(hipSetDevice(d->device));
    const int rc = wait_stream(d, timeout_ms, true);
    return rc ? rc : trpo_dev_comm_error(d);
}

// Give up on the attached collective: RCCL's abort (its kernels, eager or inside a captured graph, see
// the abort flag and exit), or the peer exchange's error word (later exchanges skip their waits); the
// CG graph holding the old collective is dropped, the stream drained (bounded), and every later result
// call of this context reports -4.  The context is then only good for trpo_ctx_destroy.
extern "C" int trpo_dev_comm_abort(trpo_dev *d) {
    if (!d) return -1;
    hipSetDevice(d->device);
    if (d->comm) {
        ncclCommAbort(d->comm);
        d->comm = NULL;
    }
    if (d->peer) trpo_peer_set_error(d->peer);
    d->comm_aborted = 1;
    const int rc = wait_stream(d, 10000, false);
    if (d->cg_exec) {
        hipGraphExecDestroy(d->cg_exec);
        d->cg_exec = NULL;
    }
    return rc;
}

// Self-check of the attached collective before it carries results: ONE eager all-reduce, through the
// same allreduce() every FVP uses, of a vector as long as the per-FVP message (Rc x Ps replica values
// in the atomic mode, the reduced vector otherwise).  Rank r contributes 2^r (1 + i mod 251) at
// element i, so the sum is (2^world - 1)(1 + i mod 251) exactly, and a lost, doubled or misplaced
// contribution changes it.  The wait is bounded (timeout_ms); every element is compared bit for bit.
// Returns 0, -6 (no completion: the caller aborts), -7 (wrong sum; *bad = mismatching elements) or the
// collective's error.  TRPO_COMM_FAULT=verify:R / hang:R (testing) makes rank R contribute a wrong
// value / skip the all-reduce.
static int comm_fault(const trpo_dev *d, const char *kind) {
    const char *e = getenv("TRPO_COMM_FAULT");
    const size_t k = strlen(kind);
    const int hit = e && !strncmp(e, kind, k) && e[k] == ':' && atoi(e + k + 1) == d->rank;
    if (hit)            // a test-only hook: never silent when it fires
        fprintf(stderr, "[trpo_mi355x] WARNING: TRPO_COMM_FAULT=%s is set: rank %d %s its self-check "
                        "all-reduce on purpose (fault injection for tests)\n", e, d->rank,
                !strcmp(kind, "hang") ? "skips" : "corrupts");
    return hit;
}

extern "C" int trpo_dev_comm_verify(trpo_dev *d, long timeout_ms, long *bad) {
    if (bad) *bad = 0;
    if (!d) return -1;
    if (d->comm_aborted) return -4;
    if (!has_collective(d)) return 0;
    HCHK(hipSetDevice(d->device));
    const size_t count = d->atomic ? (size_t)d->Rc * d->Ps : (size_t)d->nw;
    // a buffer that exists already (no allocation while another rank's exchange may be waiting):
    // the atomic sink set (never consumed) or the slab-path reduced vector (rewritten by every FVP)
    double *buf = d->atomic ? d->pacc + (long)d->R * d->Ps : d->zacc;
    if (const int hrc = ensure_hst(d, count, true)) return hrc;
    for (size_t i = 0; i < count; ++i) d->hst[i] = ldexp((double)(1 + i % 251), d->rank);
    if (comm_fault(d, "verify")) d->hst[0] += 1.0;
    hipLaunchKernelGGL(vcopy64_kernel, dim3(cdiv((long)count, 256)), dim3(256), 0, d->stream,
                       (const double *)d->hst_dev, buf, (int)count);
    HCHK(hipGetLastError());
    int rc = comm_fault(d, "hang") ? 0 : allreduce(d, buf, count);
    if (rc) return rc;
    hipLaunchKernelGGL(vcopy64_kernel, dim3(cdiv((long)count, 256)), dim3(256), 0, d->stream, (const double *)buf,
                       d->hst_dev, (int)count);
    HCHK(hipGetLastError());
    rc = wait_stream(d, timeout_ms, false);
    d->hst_pending = 0;
    if (rc) return rc;
    rc = trpo_dev_comm_error(d);
    if (rc) return rc;
    const double f = ldexp(1.0, d->world) - 1.0;
    long nbad = 0;
    for (size_t i = 0; i < count; ++i) nbad += d->hst[i] != f * (double)(1 + i % 251);
    if (bad) *bad = nbad;
    return nbad ? -7 : 0;
}

// ---------------------------------------------------------------------------
// Peer-window exchange (trpo_peer.hip).  Two steps, like RCCL's unique id: every rank opens its
// window and hands the exported handle to the caller's bootstrap; then every rank attaches with the
// world's handles in rank order (or, for contexts of one process, their window pointers).  Attaching
// replaces an RCCL communicator or host group: all collectives of the context then go through the
// exchange kernel.  All ranks must attach concurrently (the attach all-reduces the shard sizes).
// ---------------------------------------------------------------------------
static size_t peer_slot_doubles(const trpo_dev *d) {
    size_t s = (size_t)d->R * d->Ps;                       // a standalone FVP's replica sets
    if (s < (size_t)d->P + 1) s = (size_t)d->P + 1;        // the policy-gradient sums
    if (s < 64) s = 64;                                    // line-search sums, shard sizes
    return s;
}

// Round 4 refused the peer exchange under any HIP runtime but the one the library was built against: under
// the ROCm 7.0 copy a PyTorch wheel bundles, contexts created AFTER peer-attached contexts had run and been
// destroyed computed wrong FVPs.  Round 5 found the trigger -- returning the uncached peer window to that
// runtime (hipFree); none of the later contexts' own buffers reuses the freed range and no kernel reads
// memory the library never wrote (profiles/r05_peer_diag/) -- and trpo_peer.hip now keeps uncached windows
// for the life of the process (a pool reused by later peer contexts), so the exchange runs under either
// runtime (tests/test_gpu_peer.py::test_peer_slab_paths_torch_runtime_first).
extern "C" int trpo_dev_peer_open(trpo_dev *d, void *handle64) {
    if (!d) return -1;
    HCHK(hipSetDevice(d->device));
    if (!d->peer) {
        d->peer = trpo_peer_create(d->device, peer_slot_doubles(d));
        if (!d->peer) return -2;
        HCHK(trpo_malloc((void **)&d->zred, sizeof(double) * 2 * d->Ps));
        HCHK(hipMemset(d->zred, 0, sizeof(double) * 2 * d->Ps));
        HCHK(trpo_malloc((void **)&d->ptmp, sizeof(double) * trpo_peer_slot(d->peer)));
        HCHK(trpo_malloc((void **)&d->pn, sizeof(double) * PEER_WMAX));
    }
    return handle64 ? trpo_peer_handle(d->peer, handle64) : 0;
}

extern "C" void *trpo_dev_peer_window(trpo_dev *d) { return d && d->peer ? trpo_peer_window(d->peer) : NULL; }

extern "C" int trpo_dev_comm_error(const trpo_dev *d);
extern "C" int trpo_dev_set_peers(trpo_dev *d, int rank, int world, const void *handles, void *const *local) {
    if (!d || !d->peer || world < 1 || world > PEER_WMAX || rank < 0 || rank >= world) return -1;
    HCHK(hipSetDevice(d->device));
    DSYNC(d);
    const int rc = trpo_peer_connect(d->peer, rank, world, handles, local, d->stream);
    if (rc) return rc;
    if (d->comm) {
        ncclCommDestroy(d->comm);
        d->comm = NULL;
    }
    d->group = NULL;
    d->peer_on = world > 1;
    d->rank = rank;
    d->world = world;
    // contexts of ONE process sharing a device: the CG runs eagerly -- instantiating a graph may
    // allocate (and wait for the device) while another rank's exchange already spins for this one
    if (local) d->no_graph = 1;
    if (d->cg_exec) {
        hipGraphExecDestroy(d->cg_exec);
        d->cg_exec = NULL;
    }
    const int rn = refresh_n_total(d);
    return rn ? rn : trpo_dev_comm_error(d);
}

// -4 after a peer exchange whose wait timed out (a rank missing) or an abort; 0 otherwise.  A timed-out
// exchange's records (rank, workgroup, exchange, missing peer, tag seen) go to stderr the first time.
extern "C" int trpo_dev_comm_error(const trpo_dev *d) {
    if (d && d->comm_aborted) return -4;
    if (!(d && d->peer_on && trpo_peer_error(d->peer))) return 0;
    trpo_peer_report(d->peer);
    return -4;
}

extern "C" const char *trpo_hip_runtime_path(void) {
    Dl_info info;
    if (dladdr(reinterpret_cast<void *>(&hipGetDeviceCount), &info) && info.dli_fname) return info.dli_fname;
    return "";
}

extern "C" const char *trpo_dev_comm_backend(const trpo_dev *d) {
    if (!d) return "";
    if (d->comm_aborted) return "aborted";
    if (d->peer_on)
        return trpo_peer_proto(d->peer) != 1 && d->world <= 8 ? "peer-xgmi (uncached window, tagged granules)"
                                                                : "peer-xgmi (uncached window, fenced hand-off)";
    if (d->comm) return "rccl";
    if (d->group) return "host-group";
    return "none";
}

// Host <-> device vector moves through a pinned, device-mapped host buffer and a copy kernel: a
// pageable hipMemcpyAsync costs ~20 us per call (staged through a driver bounce buffer), this ~5.
__global__ void vcopy64_kernel(const double *__restrict__ src, double *__restrict__ dst, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[i];
}
// the upload of a direction for the cooperative kernel: the natural-order copy, and the same values in the
// fp32 fragment-order pack (slot pslot[i], -1 for LogStd), so the FVP loads the pack coalesced instead of
// every block gathering it (round 5; the CG's cg_axpy does the same for p')
__global__ void vcopy_pack_kernel(const double *__restrict__ src, double *__restrict__ dst, int n,
                                  float *__restrict__ vpk, const int *__restrict__ pslot) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const double v = src[i];
        dst[i] = v;
        const int s = pslot[i];
        if (s >= 0) vpk[s] = (float)v;
    }
}
// host_writes: the caller is about to write the buffer from the host (an upload); device-side
// writers (downloads) are ordered after a pending upload's copy by the stream and need no wait
// (its return code is passed on unchanged: -4 when the wait it needed found the collective failed)
// The wait of the calls whose results come back through the pinned staging buffer (copy kernels, no
// hipMemcpy to pageable memory pending): without a collective a stream write of a sequence number into
// pinned memory behind the enqueued work and a spin on it -- ~2.5 us sooner than hipStreamSynchronize per
// host round trip (tools/micro/host_wait: 9.1 vs 11.6 us for one small launch; profiles/r06_host_wait.log);
// the stream is queried after 2 ms, so a failed launch still returns its error.  Where the write is
// refused, and with a collective, trpo_dev_wait_done.
static int wait_staged(trpo_dev *d) {
    if (!has_collective(d) && d->wflag_dev) {
        if (++d->wseq == 0) d->wseq = 1;
        if (hipStreamWriteValue32(d->stream, d->wflag_dev, d->wseq, 0) == hipSuccess)
            return trpo_wait_host_flags(d->stream, d->wflag, 1, d->wseq, 2000);
    }
    return trpo_dev_wait_done(d);
}
#define DSYNC_STAGED(d)                            \
    do {                                           \
        const int dsync_rc_ = wait_staged(d);      \
        if (dsync_rc_) return dsync_rc_;           \
    } while (0)

static int ensure_hst(trpo_dev *d, size_t count, bool host_writes = false) {
    if (d->hst_pending && (host_writes || count > d->hst_cap || !d->hst)) {
        DSYNC_STAGED(d);
        d->hst_pending = 0;
    }
    if (count <= d->hst_cap && d->hst) return 0;
    if (d->hst) hipHostFree(d->hst);
    d->hst = d->hst_dev = NULL;
    d->hst_cap = 0;
    HCHK(hipHostMalloc((void **)&d->hst, sizeof(double) * count, TRPO_HOST_COHERENT));
    HCHK(hipHostGetDevicePointer((void **)&d->hst_dev, d->hst, 0));
    d->hst_cap = count;
    return 0;
}

extern "C" int trpo_dev_upload(trpo_dev *d, int slot, const double *host) {
    if (!d || slot < 0 || slot > 4 || !host) return -1;
    HCHK(hipSetDevice(d->device));
    if (const int hrc = ensure_hst(d, (size_t)d->P + 2 * (size_t)(d->hist_cap + 8), true)) return hrc;
    memcpy(d->hst, host, sizeof(double) * d->P);
    if (slot == TRPO_VEC_V && d->coop_pk) {
        hipLaunchKernelGGL(vcopy_pack_kernel, dim3(cdiv(d->P, 256)), dim3(256), 0, d->stream,
                           (const double *)d->hst_dev, d->vec[slot], d->P, (float *)d->vpack, (const int *)d->pslot);
        d->vpack_v = 1;
    } else {
        hipLaunchKernelGGL(vcopy64_kernel, dim3(cdiv(d->P, 256)), dim3(256), 0, d->stream, (const double *)d->hst_dev,
                           d->vec[slot], d->P);
    }
    HCHK(hipGetLastError());
    // no wait here: the stream orders the copy before every later kernel, and the next host-side
    // write to the staging buffer (ensure_hst) waits for it
    d->hst_pending = 1;
    return 0;
}

extern "C" int trpo_dev_download(trpo_dev *d, int slot, double *host) {
    if (!d || slot < 0 || slot > 4 || !host) return -1;
    HCHK(hipSetDevice(d->device));
    if (const int hrc = ensure_hst(d, (size_t)d->P + 2 * (size_t)(d->hist_cap + 8))) return hrc;
    hipLaunchKernelGGL(vcopy64_kernel, dim3(cdiv(d->P, 256)), dim3(256), 0, d->stream, (const double *)d->vec[slot],
                       d->hst_dev, d->P);
    HCHK(hipGetLastError());
    DSYNC_STAGED(d);
    d->hst_pending = 0;
    memcpy(host, d->hst, sizeof(double) * d->P);
    return trpo_dev_comm_error(d);
}

// x (slot X) and what the fp32 stall guard reads of the last solve -- ctl->iter, ctl->orth, alpha[] and
// the rdotr history -- in one synchronisation
extern "C" int trpo_dev_download_x_cg(trpo_dev *d, double *host, double *stats, double *rdotr, size_t cap,
                                      size_t *iters) {
    if (!d || !host || !stats || !rdotr || !iters) return -1;
    HCHK(hipSetDevice(d->device));
    const int cw = (int)cdiv(sizeof(Ctl), sizeof(double)), hw = 2 * d->hist_cap;
    if (const int hrc = ensure_hst(d, (size_t)d->P + cw + hw)) return hrc;
    hipLaunchKernelGGL(vcopy64_kernel, dim3(cdiv(d->P, 256)), dim3(256), 0, d->stream,
                       (const double *)d->vec[TRPO_VEC_X], d->hst_dev, d->P);
    hipLaunchKernelGGL(vcopy64_kernel, dim3(cdiv(cw, 256)), dim3(256), 0, d->stream, (const double *)d->ctl,
                       d->hst_dev + d->P, cw);
    if (hw) hipLaunchKernelGGL(vcopy64_kernel, dim3(cdiv(hw, 256)), dim3(256), 0, d->stream,
                               (const double *)d->hist, d->hst_dev + d->P + cw, hw);
    HCHK(hipGetLastError());
    DSYNC_STAGED(d);
    d->hst_pending = 0;
    memcpy(host, d->hst, sizeof(double) * d->P);
    Ctl c;
    memcpy(&c, d->hst + d->P, sizeof c);
    stats[0] = c.orth;
    memcpy(stats + 1, c.alpha, sizeof(double) * CG_AMAX);
    *iters = (size_t)c.iter;
    for (size_t k = 0; k <= (size_t)c.iter && k < cap && (int)k < d->hist_cap; ++k)
        rdotr[k] = d->hst[d->P + cw + 2 * k];
    return trpo_dev_comm_error(d);
}

// what a twin context needs to rebuild this one's problem (the host layer's fp64 re-solve)
extern "C" int trpo_dev_device(const trpo_dev *d) { return d ? d->device : -1; }
extern "C" int trpo_dev_is_f64(const trpo_dev *d) { return d ? d->f64 : 0; }
extern "C" int trpo_dev_get_obs(trpo_dev *d, double *host) {
    if (!d || (!host && d->n)) return -1;
    if (!d->n) return 0;
    HCHK(hipSetDevice(d->device));
    HCHK(hipMemcpyAsync(host, d->obs64, sizeof(double) * d->n * d->net.L[0], hipMemcpyDeviceToHost, d->stream));
    DSYNC(d);
    return 0;
}
extern "C" int trpo_dev_get_std(trpo_dev *d, double *host) {
    if (!d || !host) return -1;
    HCHK(hipSetDevice(d->device));
    HCHK(hipMemcpyAsync(host, d->std64, sizeof(double) * d->net.A, hipMemcpyDeviceToHost, d->stream));
    DSYNC(d);
    return 0;
}

static IterArgs plain_args(trpo_dev *d, const int *skip) {
    IterArgs a;
    memset(&a, 0, sizeof a);
    a.obs4 = reinterpret_cast<const float4 *>(d->obs4);
    a.n = (int)d->n;
    a.ntiles = cdiv((long)d->n, 16);
    a.P = d->P;
    a.Ps = d->Ps;
    a.nw = d->nw;
    a.tpack = (const float *)d->tpack;      // fp64 mode: the kernel reinterprets (element type T)
    a.vpack = (const float *)d->vpack;
    a.slabs = (float *)d->slabs;
    a.vmap = d->vmap;
    a.pslot = d->pslot;
    a.islot = d->islot;
    a.imap = d->imap;
    a.skip = skip;
    a.R_out = 1;
    a.R_in = 1;
    a.gmaj = d->gmaj_on;
    return a;
}

// block partials (fp32, or fp64 in the fp64 mode) -> d->zacc, fixed order; with zout the FVP
// epilogue (z = sum / N + damping v, log-std block 2 v + damping v) is applied on the way
// (grid: the producing launch's block count, default the CG grid)
static void launch_reduce(trpo_dev *d, const int *skip, const double *vin = nullptr, double *zout = nullptr,
                          double *zh = nullptr, int grid = 0) {
    const int G = grid > 0 ? grid : d->grid;
    if (d->f64)
        hipLaunchKernelGGL(reduce_slabs_kernel<double>, dim3(d->slab / RS_POS), dim3(RS_THREADS), 0, d->stream,
                           (const double *)d->slabs, G, d->slab, d->imap, d->zacc, skip, vin, zout, d->ctl,
                           d->nw, d->P, zh);
    else
        hipLaunchKernelGGL(reduce_slabs_kernel<float>, dim3(d->slab / RS_POS), dim3(RS_THREADS), 0, d->stream,
                           (const float *)d->slabs, G, d->slab, d->imap, d->zacc, skip, vin, zout, d->ctl,
                           d->nw, d->P, zh);
}

// a standalone (never skipped) tile-kernel FVP: the first one after theta / the observations
// changed writes the forward-activation cache (MODE 0), later ones read it (MODE 2)
static int allreduce(trpo_dev *d, double *buf, size_t count);

// Returns the atomic replica set it accumulated into (atomic mode) or NULL (block slabs: d->grid_fvp of
// them, the FVP-call grid and tile order).
// sink: a kernel-only launch whose result is never consumed (timing): accumulates into the sink set.
static double *launch_fvp_plain(trpo_dev *d, IterArgs &a, bool sink = false) {
    double *acc = NULL;
    a.gmaj = d->gmaj_fvp;
    if (d->atomic) {
        // fp64 atomics into R replicas, like the CG kernels (no slab round trip through HBM); the
        // set is zero on entry because its consumer, acc_epilogue_kernel, leaves it zeroed
        acc = d->pacc + (sink ? (long)d->R * d->Ps : 0);
        a.acc_out = acc;
        a.R_out = d->Rc;
    }
    if (d->yc_on) {
        a.yc = reinterpret_cast<float4 *>(d->yc);
        (d->yc_valid ? d->k_fvp_yc : d->k_fvp)(dim3(d->grid_fvp), d->k_lds, d->stream, a, d->net);
        d->yc_valid = 1;
    } else {
        d->k_fvp(dim3(d->grid_fvp), d->k_lds, d->stream, a, d->net);
    }
    return acc;
}

// the generic kernel on the context's element type (d->gv already holds the direction)
static void launch_generic(trpo_dev *d, const int *skip) {
    if (d->f64)
        hipLaunchKernelGGL(fvp_generic_kernel<double>, dim3(d->grid), dim3(GEN_T), 0, d->stream,
                           (const double *)d->gobs, (int)d->n, (const double *)d->gth, (const double *)d->gv,
                           (const double *)d->giv, (double *)d->scratch, d->srows, (double *)d->slabs, d->slab, d->net,
                           skip);
    else
        hipLaunchKernelGGL(fvp_generic_kernel<float>, dim3(d->grid), dim3(GEN_T), 0, d->stream,
                           (const float *)d->gobs, (int)d->n, (const float *)d->gth, (const float *)d->gv,
                           (const float *)d->giv, (float *)d->scratch, d->srows, (float *)d->slabs, d->slab, d->net,
                           skip);
}

// enqueue: partial sums of F*src into d->zacc (global over ranks)
static int enqueue_fvp_core(trpo_dev *d, const double *src, const int *skip) {
    const Net &n = d->net;
    if (d->fast) {
        // src has already been packed into d->vpack (by the caller or the CG kernels)
        IterArgs a = plain_args(d, skip);
        if (skip == &d->ctl->zero && !d->atomic) {
            launch_fvp_plain(d, a);
            launch_reduce(d, skip, nullptr, nullptr, nullptr, d->grid_fvp);
        } else {
            d->k_fvp(dim3(d->grid), d->k_lds, d->stream, a, n);
            launch_reduce(d, skip);
        }
        HCHK(hipGetLastError());
        return allreduce(d, d->zacc, d->nw);
    } else {
        hipLaunchKernelGGL(to_elem_kernel, dim3(cdiv(d->P, 256)), dim3(256), 0, d->stream, d->gv, src, (long)d->P,
                           d->f64);
        launch_generic(d, skip);
        HCHK(hipGetLastError());
    }
    launch_reduce(d, skip);
    HCHK(hipGetLastError());
    return allreduce(d, d->zacc, d->nw);
}

// z = F src into slot Z (src: any device P-vector, e.g. slot X for the update's FVP(x)); with
// *zh != NULL the atomic-replica epilogue also writes z there (mapped host memory), otherwise
// *zh is cleared and the caller downloads slot Z itself
static int fvp_src(trpo_dev *d, const double *src, double **zh) {
    if (!d || !src) return -1;
    if (d->n_total <= 0) return -1;
    HCHK(hipSetDevice(d->device));
    double *zhost = *zh;
    *zh = NULL;
    if (d->fast && (d->atomic || !has_collective(d))) {
        // two launches: the tile kernel gathers its direction fragments from v itself, then the
        // atomic-replica or slab reduce applies the epilogue (under RCCL after the all-reduce)
        IterArgs a = plain_args(d, &d->ctl->zero);
        a.v_nat = (d->coop_pk && d->vpack_v && src == d->vec[TRPO_VEC_V]) ? nullptr : src;   // packed at upload
        double *acc = launch_fvp_plain(d, a);
        if (acc) {
            if (allreduce(d, acc, (size_t)d->Rc * d->Ps)) return -4;
            hipLaunchKernelGGL(acc_epilogue_kernel, dim3(cdiv(d->P, 256)), dim3(256), 0, d->stream, acc, d->Rc,
                               src, d->vec[TRPO_VEC_Z], d->P, d->Ps, d->nw, d->ctl, zhost);
            *zh = zhost;
        } else {
            launch_reduce(d, &d->ctl->zero, src, d->vec[TRPO_VEC_Z], zhost, d->grid_fvp);
            *zh = zhost;
        }
        HCHK(hipGetLastError());
        return 0;
    }
    if (d->fast) {
        hipLaunchKernelGGL(gather_pack_kernel, dim3(cdiv(d->pack.vlen, 256)), dim3(256), 0, d->stream, d->vpack,
                           src, d->vmap, d->pack.vlen, d->f64);
        d->vpack_v = src == d->vec[TRPO_VEC_V];
    }
    int rc = enqueue_fvp_core(d, src, &d->ctl->zero);
    if (rc) return rc;
    hipLaunchKernelGGL(fvp_epilogue_kernel, dim3(cdiv(d->P, 256)), dim3(256), 0, d->stream, d->zacc,
                       src, d->vec[TRPO_VEC_Z], d->P, d->nw, d->ctl);
    HCHK(hipGetLastError());
    return 0;
}

extern "C" int trpo_dev_fvp_src(trpo_dev *d, const double *src) {
    double *zh = NULL;
    return fvp_src(d, src, &zh);
}

extern "C" int trpo_dev_fvp(trpo_dev *d) { return d ? trpo_dev_fvp_src(d, d->vec[TRPO_VEC_V]) : -1; }

// z = F v (slot V -> slot Z) and z into host memory in one stream pass: the epilogue writes z
// through the mapped staging buffer where it can, so the call waits once
extern "C" int trpo_dev_fvp_host(trpo_dev *d, double *host) {
    if (!d || !host) return -1;
    HCHK(hipSetDevice(d->device));
    if (const int hrc = ensure_hst(d, (size_t)d->P + 2 * (size_t)(d->hist_cap + 8))) return hrc;
    double *zh = d->hst_dev;                     // ordered after a pending upload's copy by the stream
    int rc = fvp_src(d, d->vec[TRPO_VEC_V], &zh);
    if (rc) return rc;
    if (!zh) return trpo_dev_download(d, TRPO_VEC_Z, host);
    DSYNC_STAGED(d);
    d->hst_pending = 0;
    memcpy(host, d->hst, sizeof(double) * d->P);
    return 0;
}

extern "C" int trpo_dev_fvp_kernel(trpo_dev *d) {
    if (!d || d->n == 0) return -1;
    HCHK(hipSetDevice(d->device));
    if (d->fast) {
        IterArgs a = plain_args(d, &d->ctl->zero);
        a.v_nat = (d->coop_pk && d->vpack_v) ? nullptr : d->vec[TRPO_VEC_V];   // as the FVP call's launch
        launch_fvp_plain(d, a, true);                  // no epilogue follows: accumulate into the sink
    } else {
        launch_generic(d, &d->ctl->zero);
    }
    HCHK(hipGetLastError());
    return 0;
}

static int ensure_hist(trpo_dev *d, size_t maxiter) {
    if ((int)maxiter + 1 <= d->hist_cap) return 0;
    if (d->hist) hipFree(d->hist);
    d->hist = NULL;
    HCHK(trpo_malloc((void **)&d->hist, sizeof(double) * 2 * (maxiter + 1)));
    d->hist_cap = (int)maxiter + 1;
    if (d->cg_exec) {
        hipGraphExecDestroy(d->cg_exec);
        d->cg_exec = NULL;
    }
    return 0;
}

static double *acc_slot(trpo_dev *d, long j) { return d->accbuf + (j % 3) * (long)d->R * d->Ps; }
static double *zred_slot(trpo_dev *d, long j) { return d->zred + (j & 1) * (long)d->Ps; }

// the one place every collective of the library goes through: RCCL, the in-process host group, or
// nothing (one rank)
static int allreduce(trpo_dev *d, double *buf, size_t count) {
    if (d->peer_on) {
        // in place through the staging vector (the exchange kernel's output must not alias its input)
        if (count > trpo_peer_slot(d->peer)) return -1;
        // a copy kernel (stream-ordered like the exchange that follows)
        hipLaunchKernelGGL(vcopy64_kernel, dim3(cdiv((long)count, 256)), dim3(256), 0, d->stream, (const double *)buf,
                           d->ptmp, (int)count);
        HCHK(hipGetLastError());
        return trpo_peer_allreduce(d->peer, d->stream, d->ptmp, 1, 0, (int)count, buf, nullptr);
    }
    if (d->group) return hgroup_allreduce(d, buf, count);
    if (!d->comm) return 0;
    return ncclAllReduce(buf, buf, count, ncclFloat64, ncclSum, d->comm, d->stream) == ncclSuccess ? 0 : -4;
}

// per-iteration arguments of the fused CG-iteration kernel K_j beyond the CG state
// (reorthogonalisation: step j-1 -> j uses the stored basis q_0 .. q_{j-2}, capped at QCAP)
static void cg_iter_args_extra(trpo_dev *d, IterArgs &a, long j) {
    a.reorth = d->reorth;
    a.q = d->reorth ? d->qbuf : nullptr;
    a.qz = d->qzero;
    a.nq = d->reorth ? (int)(j - 1 < QCAP ? j - 1 : QCAP) : 0;
}
// the CG-iteration kernel K_j (j >= 1) of the fused paths
static fast_launch_fn cg_iter_kernel(trpo_dev *d, const IterArgs &a) {
    if (d->coop) return d->yc_on ? d->k_cg_yc : d->coop_e->launch_cg;
    if (!d->yc_on) return d->k_fvp;                       // MODE 0 with the streaming reorthogonalisation
    return d->k_cg_yc_q[qb_index(a.nq)];
}
// arguments of the last CG step (after FVP M-1) and of every step of the unfused paths
// the distributed cooperative step with no collective attached: reduce_dots_kernel replaces the slab
// reduce + cg_dots pair (with a collective the all-reduce sits between them)
static bool coop_rdots(const trpo_dev *d) { return d->coop_rdots && !d->comm && !d->group && !d->peer_on; }
static int cg_step_nq(const trpo_dev *d, long sin_iter) {
    return d->reorth ? (int)(sin_iter < QCAP ? sin_iter : QCAP) : 0;
}

// CG(maxiter) as a straight-line launch sequence (captured into a hipGraph by trpo_dev_cg).
// Fast path: init, K_0 .. K_{M-1} (K_j fuses CG step j-1 -> j with FVP j), final step.
static int enqueue_cg_body(trpo_dev *d, size_t maxiter, double resth) {
    d->vpack_v = 0;                                    // the CG kernels write the direction pack
    double *x = d->vec[TRPO_VEC_X], *b = d->vec[TRPO_VEC_B];
    const int E = cg_E(d->P);
    const int vlen = d->fast ? d->pack.vlen : 0;
    const size_t shm = d->fast ? sizeof(double) * d->P : 0;
    const int *done = &d->ctl->done;
    const long M = (long)maxiter;
    const int RP = d->Rc * d->Ps;
    // the one-wave-per-tile kernel runs the CG start inside K_0 (IterArgs::init): no init launch.
    // Its atomic target acc_slot(0) is zero on entry: zeroed at allocation and by every solve's
    // final cg_update
    const bool fused_init = d->fast && M > 0 && (!d->coop || ((d->coop_dist || d->coop_fused) && d->cinit));
    if (!fused_init)
        CG_DISPATCH(E, cg_init_kernel, dim3(1), dim3(1024), shm, d->stream, b, x, d->rbuf[0], d->pbuf[0], d->P,
                    d->ctl, d->st, d->hist, (int)maxiter, resth, d->vmap, d->vpack, vlen, d->f64,
                    d->atomic ? acc_slot(d, 0) : nullptr, d->atomic ? RP : 0, d->reorth ? d->qbuf : nullptr, d->Ps);
    if (d->fast && !d->coop) {
        for (long j = 0; j < M; ++j) {
            IterArgs a = plain_args(d, j == 0 ? &d->ctl->zero : done);
            if (j == 0) {
                a.init = 1;
                a.b_init = b;
                a.init_maxiter = (int)maxiter;
                a.init_resth = resth;
                a.p_out = d->pbuf[0];
                a.r_out = d->rbuf[0];
                a.x = x;
                a.st_out = d->st;
                a.ctl = d->ctl;
                a.hist = d->hist;
                a.reorth = d->reorth;
                a.q = d->reorth ? d->qbuf : nullptr;
            }
            if (d->atomic) {
                a.acc_out = acc_slot(d, j);
                a.R_out = d->Rc;
                a.acc_zero = acc_slot(d, j + 1);
                a.zero_len = RP;
            }
            if (j > 0) {
                const int in = (int)((j - 1) & 1), out = (int)(j & 1);
                a.update = 1;
                a.acc_in = d->atomic ? (d->peer_on ? zred_slot(d, j - 1) : acc_slot(d, j - 1)) : d->zacc;
                a.R_in = d->atomic && !d->peer_on ? d->Rc : 1;
                a.p_in = d->pbuf[in];
                a.r_in = d->rbuf[in];
                a.p_out = d->pbuf[out];
                a.r_out = d->rbuf[out];
                a.x = x;
                a.st_in = d->st + in;
                a.st_out = d->st + out;
                a.ctl = d->ctl;
                a.hist = d->hist;
                a.vmap = d->vmap;
                cg_iter_args_extra(d, a, j);
            }
            // K_0 refreshes the forward-activation cache, K_1.. read it (theta is fixed in a solve)
            if (d->yc_on) a.yc = reinterpret_cast<float4 *>(d->yc);
            (j > 0 ? cg_iter_kernel(d, a) : d->k_fvp)(dim3(d->grid), d->k_lds, d->stream, a, d->net);
            int rc;
            if (d->atomic && d->peer_on) {
                // one exchange kernel: local replica sum pushed to every peer, rank-order sum -> zred
                rc = trpo_peer_allreduce(d->peer, d->stream, acc_slot(d, j), d->Rc, d->Ps, d->Ps, zred_slot(d, j), done);
            } else if (d->atomic) {
                rc = allreduce(d, acc_slot(d, j), (size_t)RP);
            } else {
                launch_reduce(d, done);
                rc = allreduce(d, d->zacc, d->nw);
            }
            if (rc) return rc;
        }
        if (M > 0) {
            const int in = (int)((M - 1) & 1), out = (int)(M & 1);
            // the last step: x only (its r', p' and basis vector are never read -- no basis loads,
            // no reorthogonalisation of a residual that only feeds the printed history)
            if (d->P <= 2 * CGL_T && !d->no_cg_last) {
                hipLaunchKernelGGL(cg_last_kernel, dim3(1), dim3(CGL_T), 0, d->stream,
                                   d->atomic ? (d->peer_on ? zred_slot(d, M - 1) : acc_slot(d, M - 1)) : d->zacc,
                                   d->atomic && !d->peer_on ? d->Rc : 1, d->pbuf[in], d->rbuf[in], x, d->P, d->Ps,
                                   d->nw, d->ctl, d->st + in, d->st + out, d->hist,
                                   d->atomic ? acc_slot(d, 0) : nullptr, d->atomic ? RP : 0, d->f64);
            } else
            CG_DISPATCH(E, cg_update_kernel, dim3(1), dim3(1024), 0, d->stream,
                        d->atomic ? (d->peer_on ? zred_slot(d, M - 1) : acc_slot(d, M - 1)) : d->zacc,
                        d->atomic && !d->peer_on ? d->Rc : 1, d->pbuf[in], d->rbuf[in],
                        (double *)nullptr, (double *)nullptr, x, d->P, d->nw, d->ctl, d->st + in, d->st + out,
                        d->hist, (const int *)nullptr, (void *)nullptr, 0, 0, (void *)nullptr,
                        (const void *)d->qzero, 0, d->Ps, d->atomic ? acc_slot(d, 0) : nullptr,
                        d->atomic ? RP : 0);
        }
    } else if (d->coop && d->coop_dist) {
        // cooperative kernel, distributed CG step: FVP j (direction gathered from p_j; K_0 recomputes
        // the forward pass and writes the cache, K_1.. read it), the slab reduce [+ all-reduce], then
        // the step over natural-order slices (cg_dots_kernel, cg_axpy_kernel)
        const int G = cdiv(d->Ps / 2, CGS_T);
        for (long j = 0; j < M; ++j) {
            const int cur = (int)(j & 1), nxt = (int)((j + 1) & 1);
            // K_0 runs even when cg_init found the solve already converged: it is what refreshes the
            // forward-activation cache that trpo_dev_ycache_written() then marks valid
            IterArgs a = plain_args(d, j == 0 ? &d->ctl->zero : done);
            a.v_nat = d->pbuf[cur];
            if (j == 0 && fused_init) {                    // the CG start inside K_0 (v = p_0 = b)
                a.v_nat = b;
                a.init = 1;
                a.b_init = b;
                a.init_maxiter = (int)maxiter;
                a.init_resth = resth;
                a.p_out = d->pbuf[0];
                a.r_out = d->rbuf[0];
                a.x = x;
                a.st_out = d->st;
                a.ctl = d->ctl;
                a.hist = d->hist;
                a.reorth = d->reorth;
                a.q = d->reorth ? d->qbuf : nullptr;
            }
            // fp32: K_j (j >= 1) reads p_j from the fragment-order pack the previous cg_axpy wrote (PK)
            if (j > 0 && !d->f64 && d->coop_pk) a.v_nat = nullptr;
            if (d->yc_on) a.yc = reinterpret_cast<float4 *>(d->yc);
            (j > 0 && d->yc_on ? d->k_fvp_yc : d->k_fvp)(dim3(d->grid), d->k_lds, d->stream, a, d->net);
            const int nq = cg_step_nq(d, j);
            void *qb = d->reorth ? d->qbuf : (void *)d->qzero;
            if (coop_rdots(d)) {                            // one rank: the reduce and the dots in one launch
                const int GR = d->slab / RS_POS;
                hipLaunchKernelGGL(reduce_dots_kernel<float>, dim3(GR), dim3(RS_THREADS), 0, d->stream,
                                   (const float *)d->slabs, d->grid, d->slab, d->imap, d->zacc, d->pbuf[cur],
                                   d->rbuf[cur], x, d->zbuf, d->dotsbuf, (const void *)qb, (const void *)d->qzero,
                                   d->reorth ? nq : 0, d->P, d->Ps, d->nw, d->ctl, done);
                hipLaunchKernelGGL(cg_axpy_kernel<float>, dim3(G), dim3(CGS_T), 0, d->stream, d->dotsbuf, GR, d->zbuf,
                                   d->pbuf[cur], d->rbuf[cur], d->pbuf[nxt], d->rbuf[nxt], x, qb,
                                   (const void *)d->qzero, d->reorth ? nq : 0, d->reorth, d->P, d->Ps, d->ctl,
                                   d->st + cur, d->st + nxt, d->hist, done,
                                   d->coop_pk ? (float *)d->vpack : (float *)nullptr, (const int *)d->pslot);
                continue;
            }
            launch_reduce(d, done);
            int rc = allreduce(d, d->zacc, d->nw);
            if (rc) return rc;
            if (d->f64) {
                hipLaunchKernelGGL(cg_dots_kernel<double>, dim3(G), dim3(CGS_T), 0, d->stream, d->zacc, d->pbuf[cur],
                                   d->rbuf[cur], x, d->zbuf, d->dotsbuf, (const void *)qb, (const void *)d->qzero,
                                   d->reorth ? nq : 0, d->P, d->Ps, d->nw, d->ctl, done);
                hipLaunchKernelGGL(cg_axpy_kernel<double>, dim3(G), dim3(CGS_T), 0, d->stream, d->dotsbuf, G, d->zbuf,
                                   d->pbuf[cur], d->rbuf[cur], d->pbuf[nxt], d->rbuf[nxt], x, qb,
                                   (const void *)d->qzero, d->reorth ? nq : 0, d->reorth, d->P, d->Ps, d->ctl,
                                   d->st + cur, d->st + nxt, d->hist, done);
            } else {
                hipLaunchKernelGGL(cg_dots_kernel<float>, dim3(G), dim3(CGS_T), 0, d->stream, d->zacc, d->pbuf[cur],
                                   d->rbuf[cur], x, d->zbuf, d->dotsbuf, (const void *)qb, (const void *)d->qzero,
                                   d->reorth ? nq : 0, d->P, d->Ps, d->nw, d->ctl, done);
                hipLaunchKernelGGL(cg_axpy_kernel<float>, dim3(G), dim3(CGS_T), 0, d->stream, d->dotsbuf, G, d->zbuf,
                                   d->pbuf[cur], d->rbuf[cur], d->pbuf[nxt], d->rbuf[nxt], x, qb,
                                   (const void *)d->qzero, d->reorth ? nq : 0, d->reorth, d->P, d->Ps, d->ctl,
                                   d->st + cur, d->st + nxt, d->hist, done,
                                   d->coop_pk ? (float *)d->vpack : (float *)nullptr, (const int *)d->pslot);
            }
        }
    } else if (d->coop_fused) {
        // cooperative kernel: K_0 = FVP of p_0 (packed by cg_init); K_j (j >= 1) = CG step j-1 -> j
        // fused with FVP j (MODE 2); each followed by the slab reduce [+ all-reduce]
        for (long j = 0; j < M; ++j) {
            // K_0 is never skipped (see the distributed path above): it refreshes the cache
            IterArgs a = plain_args(d, j == 0 ? &d->ctl->zero : done);
            if (j == 0 && fused_init) {                    // the CG start inside K_0 (v = p_0 = b)
                a.v_nat = b;
                a.init = 1;
                a.b_init = b;
                a.init_maxiter = (int)maxiter;
                a.init_resth = resth;
                a.p_out = d->pbuf[0];
                a.r_out = d->rbuf[0];
                a.x = x;
                a.st_out = d->st;
                a.ctl = d->ctl;
                a.hist = d->hist;
                a.reorth = d->reorth;
                a.q = d->reorth ? d->qbuf : nullptr;
            }
            if (j > 0) {
                const int in = (int)((j - 1) & 1), out = (int)(j & 1);
                a.update = 1;
                a.acc_in = d->zacc;
                a.R_in = 1;
                a.p_in = d->pbuf[in];
                a.r_in = d->rbuf[in];
                a.p_out = d->pbuf[out];
                a.r_out = d->rbuf[out];
                a.x = x;
                a.st_in = d->st + in;
                a.st_out = d->st + out;
                a.ctl = d->ctl;
                a.hist = d->hist;
                cg_iter_args_extra(d, a, j);
            }
            // K_0 refreshes the forward-activation cache (fp32), K_1.. read it
            if (d->yc_on) a.yc = reinterpret_cast<float4 *>(d->yc);
            (j > 0 ? cg_iter_kernel(d, a) : d->k_fvp)(dim3(d->grid), d->k_lds, d->stream, a, d->net);
            launch_reduce(d, done);
            int rc = allreduce(d, d->zacc, d->nw);
            if (rc) return rc;
        }
        if (M > 0) {
            const int in = (int)((M - 1) & 1), out = (int)(M & 1);
            CG_DISPATCH(E, cg_update_kernel, dim3(1), dim3(1024), 0, d->stream, d->zacc, 1, d->pbuf[in], d->rbuf[in],
                        (double *)nullptr, (double *)nullptr, x, d->P, d->nw, d->ctl, d->st + in, d->st + out,
                        d->hist, (const int *)nullptr, (void *)nullptr, 0, 0, (void *)nullptr,
                        (const void *)d->qzero, 0, d->Ps);                 // the last step: x only
        }
    } else {
        // generic or cooperative kernel: FVP, reduce, [all-reduce], CG step per iteration
        for (long j = 0; j < M; ++j) {
            const int cur = (int)(j & 1), nxt = (int)((j + 1) & 1);
            int rc = enqueue_fvp_core(d, d->pbuf[cur], done);
            if (rc) return rc;
            // cooperative kernel: the update also packs p' for the next FVP (fp32 fragment order)
            CG_DISPATCH(E, cg_update_kernel, dim3(1), dim3(1024), d->coop ? shm : 0, d->stream, d->zacc, 1,
                        d->pbuf[cur], d->rbuf[cur], d->pbuf[nxt], d->rbuf[nxt], x, d->P, d->nw, d->ctl, d->st + cur,
                        d->st + nxt, d->hist, d->vmap, d->vpack, d->coop ? vlen : 0, d->f64,
                        d->reorth ? d->qbuf : nullptr, (const void *)d->qzero, cg_step_nq(d, j), d->Ps);
        }
    }
    HCHK(hipGetLastError());
    return 0;
}

// Does the CG launch sequence of enqueue_cg_body(maxiter) write the forward-activation cache?  Only
// the fused paths do, in their first FVP K_0 (launched with a.yc and with the always-zero skip flag
// &ctl->zero in all three fused paths, so it runs even when cg_init finds |b|^2 < resth); maxiter = 0
// enqueues no FVP at all, and the unfused cooperative path (TRPO_COOP_FUSED=0) runs its FVPs
// through enqueue_fvp_core without the cache.
static bool cg_writes_ycache(const trpo_dev *d, size_t maxiter) {
    if (!d->yc_on || maxiter == 0 || !d->fast) return false;
    return !d->coop || d->coop_fused || d->coop_dist;
}

// after a CG solve whose K_0 wrote the forward-activation cache it holds the current theta's
// activations, so the FVP(x) that follows may read it; otherwise the cache state is left alone (a
// stale cache stays invalid and the next standalone FVP recomputes and rewrites it)
void trpo_dev_ycache_written(trpo_dev *d) {
    if (cg_writes_ycache(d, d->cg_last_iters)) d->yc_valid = 1;
}

static int dev_cg(trpo_dev *d, size_t maxiter, double resth, bool in_sequence);
extern "C" int trpo_dev_cg(trpo_dev *d, size_t maxiter, double resth) { return dev_cg(d, maxiter, resth, false); }
// the CG of the update path's device phase: between other kernels of one submission the replayed graph
// is the cheaper form (0.169 vs 0.176 ms per armDOF_0 update, 0.614 vs 0.623 ms for 2x64, N = 50k:
// profiles/r04_launch_form_ab.log) -- no consecutive graphs there, and 11 fewer host launches
int trpo_dev_cg_in_sequence(trpo_dev *d, size_t maxiter, double resth) { return dev_cg(d, maxiter, resth, true); }
static int dev_cg(trpo_dev *d, size_t maxiter, double resth, bool in_sequence) {
    if (!d || d->n_total <= 0) return -1;
    HCHK(hipSetDevice(d->device));
    if (maxiter > 100000) return -1;
    int rc = ensure_hist(d, maxiter);
    if (rc) return rc;
    d->cg_last_iters = maxiter;
    // every solve's kernels write the direction pack (cg_axpy / the fused prologue pack p'), also when
    // the solve is a replay of the captured graph, whose host-side enqueue_cg_body ran only at capture:
    // a later FVP of slot V must re-pack V, not read the last CG direction
    d->vpack_v = 0;
    // Launch form of the solve (round 4): eager stream launches unless an RCCL communicator is attached
    // (or TRPO_CG_GRAPH=1).  A replayed hipGraph runs its 11 kernels back to back, but consecutive graph
    // launches left ~3 us of idle GPU between solves; 11 eager launches cost the host ~40 us, far less
    // than the ~95 us the GPU spends on a 50k solve, so the stream never drains: 10-iteration CG at
    // N = 50k 0.1031 -> 0.1000 ms per solve for 20 solves after 5, 0.0984 -> 0.0953 for 500 after 50
    // (profiles/r04_graph_vs_eager.log).  Under RCCL the captured graph stays: an eager solve would also
    // pay the host-side cost of ten ncclAllReduce enqueues per solve.
    const char *ng = getenv("TRPO_NO_GRAPH"), *eg = getenv("TRPO_CG_GRAPH");
    const bool graph = eg ? atoi(eg) != 0 : (d->comm != NULL || in_sequence);
    if ((ng && atoi(ng)) || d->no_graph || d->group || !graph) return enqueue_cg_body(d, maxiter, resth);
    // the graph bakes (maxiter, resth) into cg_init's arguments: key on both
    if (!d->cg_exec || d->cg_graph_iters != maxiter || d->cg_graph_resth != resth) {
        if (d->cg_exec) {
            hipGraphExecDestroy(d->cg_exec);
            d->cg_exec = NULL;
        }
        hipGraph_t graph = NULL;
        // relaxed mode: RCCL may call non-stream APIs while its collective is being captured
        HCHK(hipStreamBeginCapture(d->stream, d->comm ? hipStreamCaptureModeRelaxed : hipStreamCaptureModeThreadLocal));
        rc = enqueue_cg_body(d, maxiter, resth);
        hipError_t e = hipStreamEndCapture(d->stream, &graph);
        if (!rc && e == hipSuccess) {
            e = hipGraphInstantiate(&d->cg_exec, graph, NULL, NULL, 0);
        }
        if (graph) hipGraphDestroy(graph);
        if (rc || e != hipSuccess) {
            // capture unsupported here (e.g. by the collective library): run the same sequence
            // eagerly from now on -- identical kernels, only launch overhead differs
            fprintf(stderr, "[trpo_mi355x] CG graph capture failed (%s, rc=%d); launching eagerly\n",
                    hipGetErrorString(e), rc);
            (void)hipGetLastError();
            d->cg_exec = NULL;
            d->no_graph = 1;
            return enqueue_cg_body(d, maxiter, resth);
        }
        d->cg_graph_iters = maxiter;
        d->cg_graph_resth = resth;
    }
    HCHK(hipGraphLaunch(d->cg_exec, d->stream));
    return 0;
}

extern "C" int trpo_dev_cg_history(trpo_dev *d, double *rdotr, double *xnorm, size_t cap, size_t *iters) {
    if (!d || !d->hist) return -1;
    HCHK(hipSetDevice(d->device));
    // the control block and the whole history in one move (mapped host memory, copy kernels)
    static_assert(sizeof(Ctl) % sizeof(double) == 0, "Ctl moves as 8-byte words");
    const int cw = (int)(sizeof(Ctl) / sizeof(double)), hw = 2 * d->hist_cap;
    if (const int hrc = ensure_hst(d, (size_t)d->P + 2 * (size_t)(d->hist_cap + 8))) return hrc;
    hipLaunchKernelGGL(vcopy64_kernel, dim3(1), dim3(64), 0, d->stream, (const double *)(const void *)d->ctl,
                       d->hst_dev, cw);
    hipLaunchKernelGGL(vcopy64_kernel, dim3(cdiv(hw, 256)), dim3(256), 0, d->stream, (const double *)d->hist,
                       d->hst_dev + cw, hw);
    HCHK(hipGetLastError());
    DSYNC_STAGED(d);
    d->hst_pending = 0;
    Ctl c;
    memcpy(&c, d->hst, sizeof c);
    const size_t n = (size_t)c.iter + 1;
    if ((int)n > d->hist_cap) return -2;
    double *h = (double *)malloc(sizeof(double) * 2 * n);
    if (!h) return -3;
    memcpy(h, d->hst + cw, sizeof(double) * 2 * n);
    for (size_t i = 0; i < n && i < cap; ++i) {
        if (rdotr) rdotr[i] = h[2 * i];
        if (xnorm) xnorm[i] = h[2 * i + 1];
    }
    free(h);
    if (iters) *iters = (size_t)c.iter;
    return 0;
}

extern "C" int trpo_dev_sync(trpo_dev *d) {
    if (!d) return -1;
    HCHK(hipSetDevice(d->device));
    return trpo_dev_wait_done(d);
}

// Kernel-only timing of the fused CG-iteration kernel K_j (j >= 1: CG step j-1 -> j in the prologue,
// then FVP j) exactly as the CG graph launches it, except that everything it writes goes to private
// scratch (p, r, x, the scalar state, the history, a sink replica set) so that repeated launches
// leave the context's solve untouched and never reach the convergence exit.  Inputs are the state
// of the last solve.  Returns 1 when this context has no fused CG-iteration kernel.
static int cg_iter_kernel_only(trpo_dev *d, long j, bool init) {
    const bool fused = d->fast && (!d->coop || d->coop_fused);
    if (!fused) return 1;
    if (!d->tscr) {
        const size_t bytes = sizeof(double) * (3 * (size_t)d->P + 2 * 65) + 2 * sizeof(CgSt) + sizeof(Ctl);
        HCHK(trpo_malloc(&d->tscr, bytes));
        HCHK(hipMemsetAsync(d->tscr, 0, bytes, d->stream));
    }
    double *sp = (double *)d->tscr, *sr = sp + d->P, *sx = sr + d->P, *sh = sx + d->P;
    CgSt *sst = (CgSt *)(sh + 2 * 65);
    Ctl *sctl = (Ctl *)(sst + 2);
    if (init) {   // the scratch control block never reports convergence; the scratch state is at iteration 0
        Ctl c;
        CgSt st;
        HCHK(hipMemcpyAsync(&c, d->ctl, sizeof c, hipMemcpyDeviceToHost, d->stream));
        HCHK(hipMemcpyAsync(&st, d->st, sizeof st, hipMemcpyDeviceToHost, d->stream));
        DSYNC(d);
        c.maxiter = 1 << 30;
        c.resth = -1.0;
        c.done = 0;
        c.zero = 0;
        st.iter = 0;
        HCHK(hipMemcpyAsync(sctl, &c, sizeof c, hipMemcpyHostToDevice, d->stream));
        HCHK(hipMemcpyAsync(sst, &st, sizeof st, hipMemcpyHostToDevice, d->stream));
        DSYNC(d);
    }
    IterArgs a = plain_args(d, &sctl->zero);
    a.update = 1;
    a.p_in = d->pbuf[0];
    a.r_in = d->rbuf[0];
    a.p_out = sp;
    a.r_out = sr;
    a.x = sx;
    a.st_in = sst;
    a.st_out = sst + 1;
    a.ctl = sctl;
    a.hist = sh;
    a.vmap = d->vmap;
    if (d->atomic) {
        a.acc_in = acc_slot(d, 0);
        a.R_in = d->Rc;
        a.acc_out = d->pacc + (long)d->R * d->Ps;     // the sink set: accumulates, never consumed
        a.R_out = d->Rc;
    } else {
        a.acc_in = d->zacc;
        a.R_in = 1;
    }
    cg_iter_args_extra(d, a, j);
    if (d->yc_on) a.yc = reinterpret_cast<float4 *>(d->yc);
    cg_iter_kernel(d, a)(dim3(d->grid), d->k_lds, d->stream, a, d->net);
    HCHK(hipGetLastError());
    return 0;
}

extern "C" double trpo_dev_time(trpo_dev *d, int what, int reps, size_t maxiter, double resth) {
    if (!d || reps < 1) return -1;
    if (hipSetDevice(d->device) != hipSuccess) return -2;
    int rc = 0;
    if (what == 3) {
        // the CG-iteration kernel alone, averaged over the iterations K_1 .. K_{maxiter-1} of a solve
        // (reps launches of each); needs a solve first (its state and forward cache)
        if (maxiter < 2) return -1;
        rc = trpo_dev_cg(d, maxiter, resth);
        if (rc) return rc;
        rc = cg_iter_kernel_only(d, 1, true);
        if (rc) return rc > 0 ? -1 : rc;
        if (hipStreamSynchronize(d->stream) != hipSuccess) return -2;
        hipEventRecord(d->ev0, d->stream);
        for (long j = 1; j < (long)maxiter && !rc; ++j)
            for (int i = 0; i < reps && !rc; ++i) rc = cg_iter_kernel_only(d, j, false);
        hipEventRecord(d->ev1, d->stream);
        if (rc) return rc;
        if (hipEventSynchronize(d->ev1) != hipSuccess) return -2;
        float ms = 0;
        hipEventElapsedTime(&ms, d->ev0, d->ev1);
        return (double)ms / (reps * (double)(maxiter - 1));
    }
    // warm once (also captures the CG graph)
    if (what == 0) rc = trpo_dev_fvp_kernel(d);
    else if (what == 1) rc = trpo_dev_fvp(d);
    else rc = trpo_dev_cg(d, maxiter, resth);
    if (rc) return rc;
    if (hipStreamSynchronize(d->stream) != hipSuccess) return -2;
    hipEventRecord(d->ev0, d->stream);
    for (int i = 0; i < reps && !rc; ++i) {
        if (what == 0) rc = trpo_dev_fvp_kernel(d);
        else if (what == 1) rc = trpo_dev_fvp(d);
        else rc = trpo_dev_cg(d, maxiter, resth);
    }
    hipEventRecord(d->ev1, d->stream);
    if (rc) return rc;
    if (hipEventSynchronize(d->ev1) != hipSuccess) return -2;
    float ms = 0;
    hipEventElapsedTime(&ms, d->ev0, d->ev1);
    return (double)ms / reps;
}

extern "C" const char *trpo_dev_kernel_name(const trpo_dev *d) { return d ? d->name : ""; }


extern "C" int trpo_dev_geometry(const trpo_dev *d, int *blocks, int *threads, int *lds_bytes) {
    if (!d) return -1;
    if (blocks) *blocks = d->grid;
    if (threads) *threads = d->coop ? d->coop_e->threads : d->fast ? 64 * d->fast->waves : GEN_T;
    if (lds_bytes) *lds_bytes = d->fast ? d->k_lds : 0;
    return 0;
}

// ---------------------------------------------------------------------------
// internal accessors for trpo_update.hip (trpo_common.h)
// ---------------------------------------------------------------------------
void trpo_dev_get_view(trpo_dev *d, trpo_dev_view *v) {
    v->device = d->device;
    v->stream = d->stream;
    v->net = d->net;
    v->theta64 = d->theta64;
    v->std64 = d->std64;
    v->obs64 = d->obs64;
    v->n = d->n;
    v->n_total = d->n_total;
    v->vec_b = d->vec[TRPO_VEC_B];
    v->vec_x = d->vec[TRPO_VEC_X];
    v->vec_v = d->vec[TRPO_VEC_V];
    v->vec_z = d->vec[TRPO_VEC_Z];
    v->cg_iter = &d->ctl->iter;
    v->cg_hist = d->hist;
    v->cg_stats = &d->ctl->orth;
}

int trpo_dev_allreduce64(trpo_dev *d, double *buf, size_t count) { return allreduce(d, buf, count); }

void **trpo_dev_update_state(trpo_dev *d) { return &d->upd; }

extern "C" double trpo_dev_n_total(const trpo_dev *d) { return d ? d->n_total : 0.0; }

// ---------------------------------------------------------------------------
// policy gradient through the MFMA tile kernel (MODE 1) -- TRPO_Update path
// ---------------------------------------------------------------------------
// (Action - Mean) rows [npad][ld] in fp32 (difference taken in fp64) and Adv [npad]
template <typename T>
__global__ void pg_prep_kernel(const double *__restrict__ roll, int n, int npad, int A, int ld,
                               T *__restrict__ dm, T *__restrict__ adv) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (long)npad * ld) return;
    const int s = (int)(e / ld), j = (int)(e % ld), W = 2 * A + 1;
    dm[e] = (s < n && j < A) ? (T)(roll[(long)s * W + A + j] - roll[(long)s * W + j]) : (T)0;
    if (j == 0) adv[s] = s < n ? (T)roll[(long)s * W + 2 * A] : (T)0;
}

// 1 / sigma^2 with sigma = exp(LogStd) of the current parameters
template <typename T>
__global__ void pg_iv_kernel(const double *__restrict__ theta, int P, int A, int len, T *__restrict__ iv) {
    const int j = threadIdx.x;
    if (j < len) {
        const double es = j < A ? exp(theta[P - A + j]) : 1.0;
        iv[j] = j < A ? (T)(1.0 / (es * es)) : (T)0;
    }
}

// allocation + the rollout rows of the tile kernel's policy-gradient mode (only when the rollout
// changed); kept out of captured graphs
int trpo_dev_pg_prepare(trpo_dev *d, const double *roll64, unsigned roll_gen) {
    if (!d->fast) return 1;
    HCHK(hipSetDevice(d->device));
    const int ld = 16 * d->pack.T[3];
    const size_t npad = (size_t)cdiv((long)d->n, 16) * 16 + 16;
    if (npad > d->pg_cap) {
        if (d->pg_d) hipFree(d->pg_d);
        if (d->pg_adv) hipFree(d->pg_adv);
        d->pg_d = d->pg_adv = NULL;
        d->pg_cap = 0;
        HCHK(trpo_malloc((void **)&d->pg_d, d->esz * npad * ld));
        HCHK(trpo_malloc((void **)&d->pg_adv, d->esz * npad));
        d->pg_cap = npad;
        d->pg_gen = 0;
    }
    // the (Action - Mean) / Adv rows depend on the rollout only: rebuilt when it was re-uploaded
    // (generation 0 never matches a real upload) or the sample count changed
    const bool prep = d->pg_gen != roll_gen || d->pg_n != d->n;
    d->pg_gen = roll_gen;
    d->pg_n = d->n;
    if (!d->pg_iv) {
        HCHK(trpo_malloc((void **)&d->pg_iv, d->esz * ld));
    }
    if (prep) {
        if (d->f64)
            hipLaunchKernelGGL(pg_prep_kernel<double>, dim3(cdiv((long)npad * ld, 256)), dim3(256), 0, d->stream,
                               roll64, (int)d->n, (int)npad, d->net.A, ld, (double *)d->pg_d, (double *)d->pg_adv);
        else
            hipLaunchKernelGGL(pg_prep_kernel<float>, dim3(cdiv((long)npad * ld, 256)), dim3(256), 0, d->stream,
                               roll64, (int)d->n, (int)npad, d->net.A, ld, (float *)d->pg_d, (float *)d->pg_adv);
        HCHK(hipGetLastError());
    }
    return 0;
}

int trpo_dev_pg_sums_fast(trpo_dev *d, const double *roll64, unsigned roll_gen, const double **zacc) {
    const int pr = trpo_dev_pg_prepare(d, roll64, roll_gen);
    if (pr) return pr;
    const int ld = 16 * d->pack.T[3];
    if (d->f64)
        hipLaunchKernelGGL(pg_iv_kernel<double>, dim3(1), dim3(cdiv(ld, 64) * 64), 0, d->stream, d->theta64, d->P,
                           d->net.A, ld, (double *)d->pg_iv);
    else
        hipLaunchKernelGGL(pg_iv_kernel<float>, dim3(1), dim3(cdiv(ld, 64) * 64), 0, d->stream, d->theta64, d->P,
                           d->net.A, ld, (float *)d->pg_iv);
    IterArgs a = plain_args(d, &d->ctl->zero);
    a.pg_d4 = reinterpret_cast<const float4 *>(d->pg_d);
    a.pg_adv = (const float *)d->pg_adv;
    a.pg_iv4 = reinterpret_cast<const float4 *>(d->pg_iv);
    d->k_pg(dim3(d->grid), d->k_lds, d->stream, a, d->net);
    HCHK(hipGetLastError());
    launch_reduce(d, &d->ctl->zero);
    HCHK(hipGetLastError());
    if (allreduce(d, d->zacc, d->nw)) return -4;
    *zacc = d->zacc;
    return 0;
}
