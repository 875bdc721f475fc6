/*
 * trpo_dev.h -- the thin C ABI between the C host layer (trpo_host.c) and the
 * hand-written gfx950 kernels (trpo_kernels.hip).  Plain pointers and sizes
 * only.  One trpo_dev owns everything that lives in HBM for one network and
 * one sample shard on one GPU: packed weights, observations, the CG vectors,
 * the per-block partial-sum slabs, the captured CG graph and (optionally) an
 * RCCL communicator.
 */
#ifndef TRPO_DEV_H
#define TRPO_DEV_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct trpo_dev trpo_dev;

enum { TRPO_VEC_V = 0, TRPO_VEC_Z = 1, TRPO_VEC_X = 2, TRPO_VEC_B = 3, TRPO_VEC_P = 4 };

/* device < 0: $TRPO_DEVICE or 0.  Returns NULL and fills err on failure. */
trpo_dev *trpo_dev_create(int device, size_t nl, const size_t *ls, const char *ac, char *err, size_t errlen);
/* the same with the precision forced (f64 != 0: the fp64 mode) instead of read from $TRPO_PRECISION */
trpo_dev *trpo_dev_create_prec(int device, size_t nl, const size_t *ls, const char *ac, int f64, char *err,
                               size_t errlen);
int trpo_dev_device(const trpo_dev *d);
int trpo_dev_is_f64(const trpo_dev *d);
/* copies of the problem a context holds (fp64): obs [n][L0], std [A], rollout (trpo_update.hip) */
int trpo_dev_get_obs(trpo_dev *d, double *host);
int trpo_dev_get_std(trpo_dev *d, double *host);
int trpo_dev_get_rollout(trpo_dev *d, double *mean, double *action, double *adv);
void trpo_dev_destroy(trpo_dev *d);

int trpo_dev_set_theta(trpo_dev *d, const double *theta);
int trpo_dev_set_std(trpo_dev *d, const double *stdv);
int trpo_dev_set_obs(trpo_dev *d, const double *obs, size_t n);
int trpo_dev_set_damping(trpo_dev *d, double damping);

int trpo_dev_comm_unique_id(void *id128);
/* RCCL init bounded by timeout_ms (<= 0: $TRPO_COMM_TIMEOUT_MS or 120 s); -6 on time-out */
int trpo_dev_set_comm(trpo_dev *d, int rank, int world, const void *id128, long timeout_ms);
/* bounded self-check / wait / abort of the attached collective (trpo_kernels.hip) */
int trpo_dev_comm_verify(trpo_dev *d, long timeout_ms, long *bad);
int trpo_dev_wait(trpo_dev *d, long timeout_ms);
// the closing wait of a synchronous call: hipStreamSynchronize on one rank, bounded (and the
// collective's error reported) with a collective attached
int trpo_dev_wait_done(trpo_dev *d);
#define DSYNC(d)                                     \
    do {                                             \
        const int dsync_rc_ = trpo_dev_wait_done(d); \
        if (dsync_rc_) return dsync_rc_;             \
    } while (0)
int trpo_dev_comm_abort(trpo_dev *d);
/* in-process host-staged group of `world` contexts (one thread each): the sharded code path
 * without RCCL, for tests (trpo_kernels.hip) */
typedef struct trpo_hgroup trpo_hgroup;
trpo_hgroup *trpo_hgroup_create(int world);
void trpo_hgroup_destroy(trpo_hgroup *g);
int trpo_dev_set_group(trpo_dev *d, trpo_hgroup *g, int rank);
int trpo_dev_comm_info(const trpo_dev *d, int *rank, int *world, int *replicas);
/* peer-window exchange over xGMI (trpo_peer.hip): open the own window (its 64-byte IPC handle into
 * handle64 when non-NULL), then attach with the world's handles (rank order) or, in one process,
 * the contexts' window pointers; replaces RCCL / the host group for this context */
int trpo_dev_peer_open(trpo_dev *d, void *handle64);
void *trpo_dev_peer_window(trpo_dev *d);
int trpo_dev_set_peers(trpo_dev *d, int rank, int world, const void *handles, void *const *local);
int trpo_dev_comm_error(const trpo_dev *d);
const char *trpo_dev_comm_backend(const trpo_dev *d);

int trpo_dev_upload(trpo_dev *d, int slot, const double *host);
int trpo_dev_download(trpo_dev *d, int slot, double *host);
/* x and the last CG solve's statistics, one synchronisation: stats[0] = the largest fraction of a new
 * residual the reorthogonalisation removed (0 without it), stats[1 + k] = alpha_k, k < 64; rdotr[0..iters]
 * the residual history (cap entries at most) */
#define TRPO_CG_STATS 65
int trpo_dev_download_x_cg(trpo_dev *d, double *host, double *stats, double *rdotr, size_t cap, size_t *iters);

int trpo_dev_fvp(trpo_dev *d);                 /* enqueue z = F v  (slots V -> Z) */
int trpo_dev_fvp_src(trpo_dev *d, const double *src);   /* enqueue z = F src (any device vector) -> Z */
int trpo_dev_fvp_host(trpo_dev *d, double *host); /* z = F v (V -> Z) and z -> host, one wait */
int trpo_dev_fvp_kernel(trpo_dev *d);         /* enqueue the dominant kernel alone */
int trpo_dev_cg(trpo_dev *d, size_t maxiter, double resth); /* enqueue CG on slot B -> X */
int trpo_dev_cg_history(trpo_dev *d, double *rdotr, double *xnorm, size_t cap, size_t *iters);
int trpo_dev_sync(trpo_dev *d);
/* what: 0 FVP kernel, 1 full FVP, 2 CG(maxiter) -- average ms over reps */
double trpo_dev_time(trpo_dev *d, int what, int reps, size_t maxiter, double resth);

/* TRPO_Update path (src/TRPO_Update.c), fp64.  Rollout = per local sample Mean[A],
 * Action[A], Adv.  policy_gradient leaves b in slot B (and copies it / the global
 * sum of Adv to the host when non-NULL); surrogate returns the global sums
 * sum_n Adv exp(LLD) for candidates theta + 2^-k fullstep, k = k0 .. k0+nk-1. */
int trpo_dev_set_rollout(trpo_dev *d, const double *mean, const double *action, const double *adv, size_t n);
int trpo_dev_policy_gradient(trpo_dev *d, double *b_host, double *adv_sum);
int trpo_dev_surrogate(trpo_dev *d, const double *fullstep, int k0, int nk, double *surr_host);
/* The device phase of one update with ONE host synchronisation: policy gradient -> slot B,
 * CG(maxiter, resth) -> slot X, FVP(x) -> slot Z; then b, x, z, sum(Adv), the CG iteration count and
 * (optional, capacity maxiter + 1) its rdotr / |x| history to the host, written by one kernel into
 * pinned host memory. */
int trpo_dev_update_solve(trpo_dev *d, size_t maxiter, double resth, double *b, double *x, double *z,
                          double *adv_sum, size_t *iters, double *rdotr_hist, double *xnorm_hist,
                          double max_kl, double *surr0, double *shs_lm, double *stats);
/* shs_lm (optional, 2): the step size shs = 0.5 x.Fx and lm = sqrt(shs / max_kl) as the device computed
 * them (fullstep = x / lm, fixed-order sum); surr0 (optional): the surrogate sum of the full step
 * theta + fullstep, the line search's first candidate, in the same synchronisation. */

/* Value-baseline objective (src/TRPO_Baseline.c), its own small device object. */
typedef struct trpo_bdev trpo_bdev;
trpo_bdev *trpo_bdev_create(int device, size_t nl, const size_t *ls, const char *ac, char *err, size_t errlen);
void trpo_bdev_destroy(trpo_bdev *b);
int trpo_bdev_set_data(trpo_bdev *b, const double *obs, const double *target, size_t n);
int trpo_bdev_eval(trpo_bdev *b, const double *theta, double *gsum, double *pred);
int trpo_bdev_eval_start(trpo_bdev *b, const double *theta, int want_pred);
int trpo_bdev_eval_finish(trpo_bdev *b, double *gsum, double *pred);

const char *trpo_dev_kernel_name(const trpo_dev *d);
int trpo_dev_geometry(const trpo_dev *d, int *blocks, int *threads, int *lds_bytes);
size_t trpo_dev_num_params(const trpo_dev *d);
double trpo_dev_n_total(const trpo_dev *d);    /* global sample count (all ranks) */

#ifdef __cplusplus
}
#endif
#endif
