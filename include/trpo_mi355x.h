/*
 * trpo_mi355x.h -- drop-in C ABI of the MI355X Fisher-vector-product /
 * conjugate-gradient path (libtrpo_mi355x.so).
 *
 * Part 1 replaces, symbol for symbol, the reference's L3 numerical core
 * declared in src/include/TRPO.h of custom-computing-ic/TRPO-Robot-Control:
 *
 *   TRPOparam      <- src/include/TRPO.h:6-49   (field-for-field identical layout)
 *   NumParamsCalc  <- src/include/TRPO.h:81     (impl. src/TRPO_Util.c:7-17)
 *   FVP            <- src/include/TRPO.h:89     (impl. src/TRPO_FVP.c:11-545)
 *   FVPFast        <- src/include/TRPO.h:93     (impl. src/TRPO_FVP.c:548-949)
 *   CG             <- src/include/TRPO.h:96     (impl. src/TRPO_CG.c:11-113)
 *   FVP_FPGA       <- src/include/TRPO.h:98     (accelerator twin, same signature)
 *   CG_FPGA        <- src/include/TRPO.h:101    (accelerator twin, same signature)
 *   TRPO_Update    <- src/include/TRPO.h:104    (impl. src/TRPO_Update.c:10-1011: policy
 *                     gradient, CG step, FVP(x) step size, backtracking line search)
 *   TRPOBaselineParam <- src/include/TRPO.h:50-77 (field-for-field identical layout)
 *   evaluate       <- src/TRPO_Baseline.c:29    (the value-baseline objective + gradient that
 *                     liblbfgs calls back, lbfgs_evaluate_t of src/include/lbfgs.h:378)
 *
 * Same prototypes, same by-value TRPOparam, same ownership (caller owns Input/b
 * and Result, fp64, length NumParamsCalc()), same return convention (elapsed
 * compute seconds >= 0, or -1 when a file cannot be opened / the request is
 * invalid), same stdout lines from CG.  Model and data still arrive by path
 * and may change between calls: the parsed, device-resident copy is cached
 * keyed on (path, size, mtime, NumSamples, layer shape).
 *
 * Part 2 is the in-memory context API the trainers need: no
 * per-call file I/O, observations uploaded once per update, P-vectors resident
 * in HBM through the whole CG solve, optional RCCL sample sharding.
 *
 * Linkage.  The library exports every Part-1 entry point TWICE: with C linkage
 * (FVPFast, CG, ...) and with C++ linkage (_Z7FVPFast9TRPOparamPdS0_m, ...;
 * csrc/trpo_cxx_abi.cpp forwards those to the C ones).  The reference's own
 * build/Makefile.cpuonly:5,11 compiles its callers with g++ against
 * src/include/TRPO.h:81-104, which has no extern "C", so an UNCHANGED caller
 * imports the mangled names and links as it is.  Included from C++, this
 * header declares the C names by default; define TRPO_MI355X_CXX_LINKAGE to
 * get the reference header's (C++-linkage) declarations of Part 1 instead.
 * evaluate() and Part 2 are C linkage either way (src/include/lbfgs.h:32-34
 * wraps the liblbfgs callback in extern "C").
 */
#ifndef TRPO_MI355X_H
#define TRPO_MI355X_H

#include <stddef.h>

#if defined(__cplusplus) && !defined(TRPO_MI355X_CXX_LINKAGE)
extern "C" {
#endif

#ifndef TRPO_H /* the reference's own TRPO.h already defines the struct */
typedef struct {
    char *ModelFile;         /* model: W[i] [in][out], B[i] per layer, LogStd */
    char *BaselineFile;      /* unused by this path */
    char *ResultFile;        /* unused by this path */
    char *DataFile;          /* per sample: Mean[A] Std[A] Obs[O] Action[A] Adv */
    size_t NumLayers;        /* e.g. 4 for [Input]->[H1]->[H2]->[Output] */
    char *AcFunc;            /* per layer: 'l' linear, 't' tanh, 's' sigmoid, 'o' 0.1x */
    size_t *LayerSize;       /* NumLayers sizes, input first */
    size_t NumSamples;
    double CG_Damping;
    size_t *PaddedLayerSize; /* FPGA only; ignored */
    size_t *NumBlocks;       /* FPGA only; ignored */
} TRPOparam;

size_t NumParamsCalc(size_t *LayerSize, size_t NumLayers);
double FVP(TRPOparam param, double *Result, double *Input);
double FVPFast(TRPOparam param, double *Result, double *Input, size_t NumThreads);
double CG(TRPOparam param, double *Result, double *b, size_t MaxIter, double ResidualTh, size_t NumThreads);
double FVP_FPGA(TRPOparam param, double *Result, double *Input);
double CG_FPGA(TRPOparam param, double *Result, double *b, size_t MaxIter, double ResidualTh, size_t NumThreads);
double TRPO_Update(TRPOparam param, double *Result, size_t NumThreads);

typedef struct {
    size_t NumLayers;
    size_t ObservSpaceDim;   /* the baseline's input is [Obs, step / EpLen]: LayerSizeBase[0] = this + 1 */
    size_t NumEpBatch;
    size_t EpLen;
    size_t NumSamples;       /* NumEpBatch * EpLen */
    size_t NumParams;        /* weights + biases (no LogStd) */
    int PaddedParams;        /* NumParams rounded up to 16 (the L-BFGS vector length) */
    char *AcFunc;
    size_t *LayerSizeBase;
    double **WBase;          /* written from x on every call, like the reference */
    double **BBase;
    double **LayerBase;      /* reference scratch; untouched */
    double **GWBase;
    double **GBBase;
    double **GLayerBase;
    double *Observ;          /* [NumSamples][ObservSpaceDim] */
    double *Target;          /* [NumSamples] */
    double *Predict;         /* [NumSamples], written on every call */
} TRPOBaselineParam;
#endif

#if defined(__cplusplus) && !defined(TRPO_MI355X_CXX_LINKAGE)
} /* extern "C" (Part 1) */
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* liblbfgs callback (double precision lbfgsfloatval_t): instance = TRPOBaselineParam*.
 * Objective 0.01 * mean((Predict - Target)^2) + 0.001 * |x[0:NumParams]|^2 and its gradient
 * (zero beyond NumParams).  Returns -1 for an unsupported activation like the reference. */
double evaluate(void *instance, const double *x, double *g, const int n, const double step);

/* ------------------------------------------------------------------------- */
/* Part 2: in-memory context API                                             */
/* ------------------------------------------------------------------------- */

typedef struct trpo_ctx trpo_ctx;

/* Error codes (negative) returned by the int-valued functions. */
enum {
    TRPO_OK = 0,
    TRPO_E_INVALID = -1,   /* bad shape, activation, NULL pointer */
    TRPO_E_DEVICE = -2,    /* no usable MI355X / HIP error */
    TRPO_E_NOMEM = -3,
    TRPO_E_COMM = -4,      /* collective failure (RCCL, peer exchange timed out, aborted) */
    TRPO_E_IO = -5,
    TRPO_E_TIMEOUT = -6,   /* a bounded wait expired (RCCL init, self-check, trpo_ctx_wait) */
    TRPO_E_VERIFY = -7     /* the collective's self-check summed wrong */
};

/* Create a context on HIP device `device` (-1: current / $TRPO_DEVICE / 0).
 * theta: flat parameters (W, B per layer, LogStd), fp64, NumParamsCalc long.
 * obs: [n][layer_size[0]] fp64 row-major (this rank's samples).
 * stdv: [layer_size[nl-1]] action std (the data file's Std column).
 * Returns NULL on failure (trpo_last_error() has the message). */
trpo_ctx *trpo_ctx_create(size_t num_layers, const size_t *layer_size, const char *acfunc,
                          const double *theta, const double *obs, size_t n, const double *stdv,
                          double cg_damping, int device);
void trpo_ctx_destroy(trpo_ctx *ctx);

int trpo_ctx_set_theta(trpo_ctx *ctx, const double *theta);
int trpo_ctx_set_obs(trpo_ctx *ctx, const double *obs, size_t n);
int trpo_ctx_set_std(trpo_ctx *ctx, const double *stdv);
int trpo_ctx_set_damping(trpo_ctx *ctx, double cg_damping);
size_t trpo_ctx_num_params(const trpo_ctx *ctx);

/* Attach an RCCL communicator: the context's samples are this rank's shard;
 * every FVP all-reduces the P-sized partial sum once (fp64, sum) and divides
 * by the GLOBAL sample count.  unique_id: 128 bytes from trpo_comm_unique_id()
 * on rank 0, broadcast by the caller. */
int trpo_comm_unique_id(void *unique_id_128);
int trpo_ctx_attach_comm(trpo_ctx *ctx, int rank, int world, const void *unique_id_128);
/* The same with RCCL's initialisation bounded: ncclCommInitRank runs in a helper thread and the call
 * returns TRPO_E_TIMEOUT when it has not completed after timeout_ms (<= 0: $TRPO_COMM_TIMEOUT_MS,
 * default 120 000) -- e.g. a rank that never calls in; the plain attach uses that default too. */
int trpo_ctx_attach_comm_timeout(trpo_ctx *ctx, int rank, int world, const void *unique_id_128, long timeout_ms);

/* In-process sharding without RCCL: `world` contexts of ONE process, each driven by its own
 * thread (any devices, the same one included), attach to a host group and run the sharded code
 * path with a host-staged all-reduce (rank-order sums: identical bits on every rank).  Meant for
 * tests and debugging of the multi-rank logic on one GPU; CG runs eagerly under a group.
 * trpo_ctx_attach_group must be called by all ranks concurrently (it all-reduces N). */
typedef struct trpo_group trpo_group;
trpo_group *trpo_group_create(int world);
void trpo_group_destroy(trpo_group *g);
int trpo_ctx_attach_group(trpo_ctx *ctx, trpo_group *g, int rank);

/* The attached communicator as the collective library reports it: this context's rank, the rank
 * count (RCCL's ncclCommCount; 1 without a communicator) and the fp64 atomic replica sets each FVP
 * all-reduces (0 when the block-slab reduction is in use). */
int trpo_ctx_comm_info(const trpo_ctx *ctx, int *rank, int *world, int *replicas);

/* Peer-window exchange over xGMI (one-shot all-reduce; no reference counterpart -- it replaces the
 * collective under the sharded CG of src/TRPO_CG.c:45-104).  Each rank allocates an exchange window
 * in its own HBM and exports it: trpo_ctx_peer_handle() writes TRPO_PEER_HANDLE_BYTES; the caller
 * all-gathers the handles (its own bootstrap, as for the RCCL unique id) and every rank calls
 * trpo_ctx_attach_peers() concurrently with the world's handles in rank order.  Every collective of
 * the context then goes through the exchange kernel (rank-order sums: identical bits on every rank);
 * the CG graph's per-FVP all-reduce is one kernel.  Contexts of ONE process (tests; any devices)
 * attach with trpo_ctx_attach_peers_local() after each has called trpo_ctx_peer_handle(ctx, NULL).
 * A rank that never arrives makes the exchange give up after 3 s: later calls return an error.
 * Attach once per context: the exchange numbering lives with the windows, so all ranks of a world
 * must be fresh contexts attached together (re-attaching one rank alone desynchronises it). */
#define TRPO_PEER_HANDLE_BYTES 64
#define TRPO_PEER_MAX_RANKS 16
int trpo_ctx_peer_handle(trpo_ctx *ctx, void *handle_64);
int trpo_ctx_attach_peers(trpo_ctx *ctx, int rank, int world, const void *handles);
int trpo_ctx_attach_peers_local(trpo_ctx *ctx, int rank, int world, trpo_ctx *const *all);
/* Self-check of the attached collective (any backend), called by ALL ranks together before it carries
 * results: one eager all-reduce, as long as the per-FVP message, of a rank-dependent test vector whose
 * exact sum is known; completion awaited at most timeout_ms (<= 0: the default above), every element
 * compared bit for bit.  0, TRPO_E_TIMEOUT (call trpo_ctx_comm_abort), TRPO_E_VERIFY or TRPO_E_COMM.
 * No reference counterpart: the reference's CG (src/TRPO_CG.c:45-104) is single-process. */
int trpo_ctx_comm_verify(trpo_ctx *ctx, long timeout_ms);
/* Wait for the context's enqueued work (e.g. trpo_ctx_enqueue_cg) at most timeout_ms: 0,
 * TRPO_E_TIMEOUT, or the collective's error. */
int trpo_ctx_wait(trpo_ctx *ctx, long timeout_ms);
/* Give up on the collective: ncclCommAbort (kernels blocked in it exit) or the peer exchange's error
 * flag, the stream drained (bounded); every later result call fails with TRPO_E_COMM.  Destroy the
 * context afterwards. */
int trpo_ctx_comm_abort(trpo_ctx *ctx);
/* "rccl", "peer-xgmi (...)", "host-group", "aborted" or "none" */
const char *trpo_ctx_comm_backend(const trpo_ctx *ctx);
/* Path of the HIP runtime (libamdhip64) this library's calls resolved to.  The library is built and
 * validated against the system ROCm (/opt/rocm); a process that loads another copy with the same
 * soname first (e.g. the one a PyTorch wheel bundles, imported before this library) makes the
 * library run on that one instead. */
const char *trpo_hip_runtime_path(void);

/* Host-pointer convenience entry points (copy in / compute / copy out).
 * Return elapsed seconds (>= 0) or a negative error code. */
double trpo_ctx_fvp(trpo_ctx *ctx, const double *v, double *out);
double trpo_ctx_cg(trpo_ctx *ctx, const double *b, size_t max_iter, double residual_th, double *x,
                   int verbose);
/* Per-iteration values CG prints: rdotr[i], |x|[i] for i = 0..iters. */
int trpo_ctx_cg_history(const trpo_ctx *ctx, double *rdotr, double *xnorm, size_t cap, size_t *iters);
/* The fp32 stall guard of the last trpo_ctx_cg / trpo_ctx_update (and the file entry points), DESIGN §3:
 * ritz_residual = the smallest relative Ritz residual of the solve's Lanczos matrix (from its CG
 * coefficients); below $TRPO_RITZ_RERUN (default 1e-14) the reference's fp64 CG loses orthogonality and
 * its step is its rounding's, so the solve was repeated in fp64 (*fp64_rerun = 1; one-rank contexts; a
 * "[WARN]" line on stderr).  orth_loss = the largest fraction of a new residual the fp32 path's
 * reorthogonalisation removed.  Any pointer may be NULL.  No reference counterpart. */
int trpo_ctx_cg_status(const trpo_ctx *ctx, double *ritz_residual, double *orth_loss, int *fp64_rerun);

/* Device-resident benchmarking hooks: b stays in HBM, no host round trip.  trpo_ctx_enqueue_cg is the
 * plain device solve: the fp32 stall guard (trpo_ctx_cg_status) never re-solves it.  After a
 * trpo_ctx_cg that the guard re-solved in fp64, slot X (trpo_ctx_download_x) holds the returned fp64 x. */
int trpo_ctx_upload_b(trpo_ctx *ctx, const double *b);
int trpo_ctx_upload_v(trpo_ctx *ctx, const double *v);
int trpo_ctx_enqueue_fvp(trpo_ctx *ctx);                                  /* z = F v */
int trpo_ctx_enqueue_cg(trpo_ctx *ctx, size_t max_iter, double residual_th); /* eager, or a graph under RCCL */
int trpo_ctx_enqueue_fvp_kernel_only(trpo_ctx *ctx);                      /* dominant kernel */
int trpo_ctx_synchronize(trpo_ctx *ctx);
/* Average duration (ms) of `reps` back-to-back launches of `what`
 * (0 = FVP kernel alone, 1 = full FVP, 2 = CG solve of max_iter), measured with
 * HIP events on the context's stream. */
double trpo_ctx_time(trpo_ctx *ctx, int what, int reps, size_t max_iter, double residual_th);
int trpo_ctx_download_x(trpo_ctx *ctx, double *x);
int trpo_ctx_download_z(trpo_ctx *ctx, double *z);

/* One TRPO policy update on the context's samples (src/TRPO_Update.c:254-1007):
 * policy gradient b from the rollout, CG (F + damping I) x = b, shs = x.Fx / 2,
 * lagrange = sqrt(shs / max_kl), fullstep = x / lagrange, backtracking line search
 * over step fractions 0.5^k (k < max_backtracks) accepting the first with
 * ratio > accept_ratio and positive improvement.  theta_out receives the new
 * parameters -- or, as in the reference, the CG step direction x itself when no
 * step fraction is accepted (src/TRPO_Update.c:850-852).  b_out / x_out / info may
 * be NULL.  Requires trpo_ctx_set_rollout() for the current samples.  verbose != 0
 * prints the reference's stdout lines (CG Iter, shs, lagrange multiplier, fval
 * before, a/e/r).  Returns elapsed seconds or a negative error code. */
#define TRPO_MAX_BACKTRACKS 32
typedef struct {
    double shs, lagrange, gnorm, fval_before, expected_improve_rate;
    int evaluated;           /* step fractions evaluated (printed) */
    int accepted;            /* accepted k (step fraction 0.5^k), or -1 */
    double actual[TRPO_MAX_BACKTRACKS], expected[TRPO_MAX_BACKTRACKS], ratio[TRPO_MAX_BACKTRACKS];
    size_t cg_iters;
} trpo_update_info;

/* Rollout of this rank's samples for the update: mean [n][A] (the policy mean the
 * actions were drawn with), action [n][A], adv [n]. */
int trpo_ctx_set_rollout(trpo_ctx *ctx, const double *mean, const double *action, const double *adv);
double trpo_ctx_update(trpo_ctx *ctx, size_t cg_max_iter, double cg_residual_th, double max_kl,
                       int max_backtracks, double accept_ratio, double *theta_out, double *b_out,
                       double *x_out, trpo_update_info *info, int verbose);
/* The line search's surrogate sums (src/TRPO_Update.c:951-981) on their own: surr[j] =
 * sum over ALL ranks' samples of Adv exp(LLD) at theta + 0.5^(k0 + j) fullstep, j < nk (nk <= 64),
 * for the context's current theta and rollout. */
int trpo_ctx_surrogate(trpo_ctx *ctx, const double *fullstep, int k0, int nk, double *surr);

/* Value-baseline context: data uploaded once per fit, then one device evaluation per L-BFGS
 * callback.  layer_size[0] = observation dim + 1 (the time feature). */
typedef struct trpo_baseline trpo_baseline;
trpo_baseline *trpo_baseline_create(size_t num_layers, const size_t *layer_size, const char *acfunc, int device);
void trpo_baseline_destroy(trpo_baseline *b);
/* observ [num_ep * ep_len][layer_size[0] - 1], target [num_ep * ep_len] */
int trpo_baseline_set_data(trpo_baseline *b, const double *observ, const double *target, size_t num_ep,
                           size_t ep_len);
/* objective at x (n >= NumParams entries, L-BFGS padding allowed); g (n) and predict (may be NULL) */
double trpo_baseline_evaluate(trpo_baseline *b, const double *x, double *g, int n, double *predict);

/* Introspection: which kernel family serves this context ("mfma-mlp3 T0xT1xT2xT3"
 * or "generic"), and the FVP launch geometry. */
const char *trpo_ctx_kernel_name(const trpo_ctx *ctx);
int trpo_ctx_launch_geometry(const trpo_ctx *ctx, int *blocks, int *threads, int *lds_bytes);

const char *trpo_last_error(void);
/* Drop every cached file-based context (FVPFast/FVP/CG cache). */
void trpo_cache_clear(void);

/* ------------------------------------------------------------------------- */
/* Part 3: the reference's text formats, as the Part-1 entry points read them */
/* ------------------------------------------------------------------------- */
/* Up to `want` doubles from whitespace-separated text with fscanf("%lf") semantics (stops at the end
 * or at the first token that is not a number); returns how many were parsed. */
size_t trpo_text_parse_doubles(const char *txt, double *out, size_t want);
/* Model file (src/TRPO_FVP.c:670-699): theta[P] (W, B per layer, then the LogStd line, which the
 * reference reads as Std); entries the file lacks are 0.  0, or -1 if it cannot be opened. */
int trpo_text_load_model(const char *path, size_t P, double *theta);
/* Data file (src/TRPO_FVP.c:731-762, src/TRPO_Update.c:228-249): the first n rows of
 * Mean[A] Std[A] Obs[O] Action[A] Adv; stdv = the LAST row's Std; mean / action / adv may be NULL. */
int trpo_text_load_data(const char *path, size_t O, size_t A, size_t n, double *obs, double *stdv, double *mean,
                        double *action, double *adv);

#ifdef __cplusplus
}
#endif
#endif /* TRPO_MI355X_H */
