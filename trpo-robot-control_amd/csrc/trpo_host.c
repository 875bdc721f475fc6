/*
 * trpo_host.c -- C host layer of libtrpo_mi355x.so.
 *
 * Implements the reference's C entry points (src/include/TRPO.h:81-101) and the
 * in-memory context API of include/trpo_mi355x.h on top of the thin device ABI
 * (csrc/trpo_dev.h).  Everything numerical runs on the GPU; this file parses
 * the reference's text formats, caches parsed + uploaded problems, keeps the
 * reference's side effects (CG progress lines, "[ERROR] ..." messages, return
 * conventions) and times the compute region the way the reference does
 * (file parsing excluded).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <math.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <sys/time.h>

#include "../../include/trpo_mi355x.h"
#include "trpo_dev.h"
#include "trpo_textio.h"

#define MAX_LAYERS 8

static __thread char g_err[512];

static void set_err(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
}

const char *trpo_last_error(void) { return g_err; }

static double now_s(void) {
    struct timeval tv;
    gettimeofday(&tv, NULL);
    return (double)tv.tv_sec + 1e-6 * (double)tv.tv_usec;
}

/* src/TRPO_Util.c:7-17 */
size_t NumParamsCalc(size_t *LayerSize, size_t NumLayers) {
    size_t p = 0;
    if (!LayerSize || NumLayers < 1) return 0;
    for (size_t i = 0; i + 1 < NumLayers; ++i) p += LayerSize[i] * LayerSize[i + 1] + LayerSize[i + 1];
    return p + LayerSize[NumLayers - 1];
}

/* ------------------------------------------------------------------------- */
/* contexts                                                                  */
/* ------------------------------------------------------------------------- */
struct trpo_ctx {
    trpo_dev *dev;
    size_t nl;
    size_t ls[MAX_LAYERS];
    char ac[MAX_LAYERS + 1];
    size_t P;
    size_t n;
    double damping;
    double *theta;             /* host copy of the current parameters (line search base) */
    int have_roll;             /* rollout uploaded for the current samples */
    trpo_dev *twin;            /* fp64 twin of the problem (the fp32 stall guard's re-solve), lazily built */
    double last_orth;          /* the last CG solve's orthogonality-loss statistic (ctl->orth) */
    double last_ritz;          /* its smallest relative Ritz residual (the stall guard's test) */
    int last_rerun;            /* 1 when the last solve's result came from the fp64 twin */
};

/* fp32 stall guard.  The fp32 path reorthogonalises every new CG residual
 * and so converges like exact-arithmetic CG.  The reference's plain fp64 recurrence
 * (src/TRPO_CG.c:65-103) does not where its residuals lose orthogonality -- which, by Paige's theory of
 * the Lanczos process, happens once a Ritz value of the solve has converged to near machine precision:
 * |q . r_k| ~ eps ||A|| / (Ritz residual).  The solve's own CG coefficients give that test: alpha_k and
 * beta_k = rdotr_{k+1} / rdotr_k form the Lanczos matrix T_k, and a Ritz pair (theta, s) of T_k has the
 * residual sqrt(beta_k) / alpha_k |s_k|.  When the smallest one, relative to the largest Ritz value,
 * falls below TRPO_RITZ_RERUN (default 1e-15, about 10 eps64) the reference's own step is its rounding's,
 * not the exact one (random-shape draw 23: 7e-17, the fp32 step 1.2e-3 from the reference; the next
 * smallest case 1.6e-15, 7e-6; tools/diag/ritz_probe.py), and the solve is repeated in fp64 on a twin of
 * the context (the reference's arithmetic, no reorthogonalisation), built on first use from the
 * context's own device-resident problem.  One rank only: a sharded context reports the statistic
 * (trpo_ctx_cg_status) and warns.  The coefficients of the fp32 trajectory carry ~1e-7 relative noise;
 * the Ritz residual is insensitive to it (the probe perturbs them: unchanged to 2 digits). */
static double ritz_threshold(void) {
    const char *e = getenv("TRPO_RITZ_RERUN");
    return e ? atof(e) : 1e-14;
}

/* eigenvalues d[] of the symmetric tridiagonal matrix (diagonal d, e[i] = T[i][i+1] for i < n - 1) and
 * the LAST components zl[] of its eigenvectors: implicit QL with Wilkinson shifts, the last row of the
 * eigenvector matrix carried alone (O(n^2)); -1 if it does not converge */
static int tql_last(double *d, double *e, double *zl, int n) {
    for (int i = 0; i < n; ++i) zl[i] = i == n - 1 ? 1.0 : 0.0;
    e[n - 1] = 0.0;
    for (int l = 0; l < n; ++l) {
        int iter = 0, m;
        do {
            for (m = l; m < n - 1; ++m) {
                const double dd = fabs(d[m]) + fabs(d[m + 1]);
                if (fabs(e[m]) <= 2.2e-16 * dd) break;
            }
            if (m != l) {
                if (iter++ == 60) return -1;
                double g = (d[l + 1] - d[l]) / (2.0 * e[l]);
                double r = hypot(g, 1.0);
                g = d[m] - d[l] + e[l] / (g + copysign(r, g));
                double sn = 1.0, cs = 1.0, p = 0.0;
                int i;
                for (i = m - 1; i >= l; --i) {
                    double f = sn * e[i];
                    const double b = cs * e[i];
                    e[i + 1] = (r = hypot(f, g));
                    if (r == 0.0) {
                        d[i + 1] -= p;
                        e[m] = 0.0;
                        break;
                    }
                    sn = f / r;
                    cs = g / r;
                    g = d[i + 1] - p;
                    r = (d[i] - g) * sn + 2.0 * cs * b;
                    d[i + 1] = g + (p = sn * r);
                    g = cs * r - b;
                    f = zl[i + 1];                       /* the last eigenvector row, rotated alone */
                    zl[i + 1] = sn * zl[i] + cs * f;
                    zl[i] = cs * zl[i] - sn * f;
                }
                if (r == 0.0 && i >= l) continue;
                d[l] -= p;
                e[l] = g;
                e[m] = 0.0;
            }
        } while (m != l);
    }
    return 0;
}

/* smallest relative Ritz residual of the Lanczos matrix T_iters of a CG solve (alpha_k, rdotr_k as the
 * device recorded them; iters <= 64); 1 when there is nothing to test.  Only the last T: a Ritz value
 * that has converged stays converged, and over the goldens and the 36 random draws the minimum over
 * T_1 .. T_iters always sat at the last one (tools/diag/ritz_probe.py); ~1 us on the host for 10 steps. */
static double ritz_min(const double *alpha, const double *rdotr, size_t iters) {
    int K = iters > 64 ? 64 : (int)iters;
    for (int j = 0; j < K; ++j)                /* the valid prefix (a converged solve stops early) */
        if (!(alpha[j] > 0.0) || !(rdotr[j] > 0.0) || !isfinite(alpha[j]) || !(rdotr[j + 1] >= 0.0)) {
            K = j;
            break;
        }
    if (K < 1) return 1.0;
    double d[64], e[64], zl[64];
    for (int j = 0; j < K; ++j) {
        d[j] = 1.0 / alpha[j] + (j > 0 ? (rdotr[j] / rdotr[j - 1]) / alpha[j - 1] : 0.0);
        e[j] = j + 1 < K ? sqrt(rdotr[j + 1] / rdotr[j]) / alpha[j] : 0.0;
    }
    if (tql_last(d, e, zl, K)) return 1.0;
    double wmax = 0.0, best = 1.0;
    for (int i = 0; i < K; ++i) wmax = fabs(d[i]) > wmax ? fabs(d[i]) : wmax;
    const double bk = sqrt(rdotr[K] / rdotr[K - 1]) / alpha[K - 1];
    for (int i = 0; i < K && wmax > 0.0; ++i) {
        const double res = bk * fabs(zl[i]) / wmax;
        best = res < best ? res : best;
    }
    return best;
}

static void drop_twin(trpo_ctx *c) {
    if (c && c->twin) {
        trpo_dev_destroy(c->twin);
        c->twin = NULL;
    }
}

/* stats = [orth, alpha_0 .. alpha_63] and the rdotr history of the solve just run */
static int needs_rerun(trpo_ctx *c, const double *stats, const double *rdotr, size_t iters) {
    c->last_orth = stats[0];
    c->last_ritz = ritz_min(stats + 1, rdotr, iters);
    const double th = ritz_threshold();
    if (!(th > 0.0) || !(c->last_ritz < th) || trpo_dev_is_f64(c->dev)) return 0;
    int world = 1;
    trpo_dev_comm_info(c->dev, NULL, &world, NULL);
    if (world > 1) {
        fprintf(stderr, "[WARN] CG: a Ritz value converged to %.1e (relative residual): the reference's fp64 CG "
                        "loses orthogonality here; sharded context, not re-solved in fp64\n", c->last_ritz);
        return 0;
    }
    return 1;
}

static trpo_dev *get_twin(trpo_ctx *c) {
    if (c->twin) return c->twin;
    char err[256] = {0};
    trpo_dev *t = trpo_dev_create_prec(trpo_dev_device(c->dev), c->nl, c->ls, c->ac, 1, err, sizeof err);
    if (!t) {
        set_err("fp64 twin: %s", err);
        return NULL;
    }
    const size_t L0 = c->ls[0], A = c->ls[c->nl - 1], n = c->n;
    double *obs = (double *)malloc(sizeof(double) * (n * L0 + 1)), *stdv = (double *)malloc(sizeof(double) * A);
    double *roll = c->have_roll ? (double *)malloc(sizeof(double) * (n * (2 * A + 1) + 1)) : NULL;
    int rc = (!obs || !stdv || (c->have_roll && !roll)) ? TRPO_E_NOMEM : trpo_dev_get_obs(c->dev, obs);
    if (!rc) rc = trpo_dev_get_std(c->dev, stdv);
    if (!rc) rc = trpo_dev_set_theta(t, c->theta);
    if (!rc) rc = trpo_dev_set_std(t, stdv);
    if (!rc) rc = trpo_dev_set_obs(t, obs, n);
    if (!rc) rc = trpo_dev_set_damping(t, c->damping);
    if (!rc && c->have_roll) {
        rc = trpo_dev_get_rollout(c->dev, roll, roll + n * A, roll + 2 * n * A);
        if (!rc) rc = trpo_dev_set_rollout(t, roll, roll + n * A, roll + 2 * n * A, n);
    }
    free(obs);
    free(stdv);
    free(roll);
    if (rc) {
        set_err("fp64 twin: rebuilding the problem failed (code %d)", rc);
        trpo_dev_destroy(t);
        return NULL;
    }
    c->twin = t;
    return t;
}

static int check_shape(size_t nl, const size_t *ls, const char *ac) {
    if (nl < 2 || nl > MAX_LAYERS || !ls || !ac) {
        set_err("unsupported NumLayers=%zu (2..%d)", nl, MAX_LAYERS);
        return -1;
    }
    for (size_t i = 0; i < nl; ++i)
        if (ls[i] == 0) {
            set_err("LayerSize[%zu] is 0", i);
            return -1;
        }
    for (size_t i = 1; i < nl; ++i)
        if (ac[i] != 'l' && ac[i] != 't' && ac[i] != 'o' && ac[i] != 's') {
            set_err("AC Function for Layer[%zu] is %c. Unsupported.", i, ac[i]);
            return -1;
        }
    return 0;
}

trpo_ctx *trpo_ctx_create(size_t num_layers, const size_t *layer_size, const char *acfunc, const double *theta,
                          const double *obs, size_t n, const double *stdv, double cg_damping, int device) {
    if (check_shape(num_layers, layer_size, acfunc)) return NULL;
    trpo_ctx *c = (trpo_ctx *)calloc(1, sizeof(trpo_ctx));
    if (!c) return NULL;
    c->nl = num_layers;
    memcpy(c->ls, layer_size, num_layers * sizeof(size_t));
    memcpy(c->ac, acfunc, num_layers);
    c->P = NumParamsCalc(c->ls, c->nl);
    char err[256] = {0};
    c->dev = trpo_dev_create(device, num_layers, layer_size, acfunc, err, sizeof err);
    if (!c->dev) {
        set_err("%s", err);
        free(c);
        return NULL;
    }
    c->theta = (double *)calloc(c->P, sizeof(double));
    if (!c->theta) {
        trpo_dev_destroy(c->dev);
        free(c);
        return NULL;
    }
    if (theta) memcpy(c->theta, theta, c->P * sizeof(double));
    if ((theta && trpo_dev_set_theta(c->dev, theta)) || (stdv && trpo_dev_set_std(c->dev, stdv)) ||
        ((obs || n == 0) && trpo_dev_set_obs(c->dev, obs, n)) || trpo_dev_set_damping(c->dev, cg_damping)) {
        set_err("device initialisation failed (theta/std/obs upload)");
        trpo_ctx_destroy(c);
        return NULL;
    }
    c->n = n;
    c->damping = cg_damping;
    return c;
}

void trpo_ctx_destroy(trpo_ctx *c) {
    if (!c) return;
    drop_twin(c);
    trpo_dev_destroy(c->dev);
    free(c->theta);
    free(c);
}

int trpo_ctx_set_theta(trpo_ctx *c, const double *theta) {
    if (!c || !theta) return TRPO_E_INVALID;
    drop_twin(c);
    int rc = trpo_dev_set_theta(c->dev, theta);
    if (!rc) memcpy(c->theta, theta, c->P * sizeof(double));
    return rc;
}
int trpo_ctx_set_obs(trpo_ctx *c, const double *obs, size_t n) {
    if (!c || (!obs && n)) return TRPO_E_INVALID;
    drop_twin(c);
    int rc = trpo_dev_set_obs(c->dev, obs, n);
    if (!rc) c->n = n;
    c->have_roll = 0;                  /* a rollout belongs to one set of samples */
    return rc;
}
int trpo_ctx_set_std(trpo_ctx *c, const double *stdv) {
    if (!c || !stdv) return TRPO_E_INVALID;
    drop_twin(c);
    return trpo_dev_set_std(c->dev, stdv);
}
int trpo_ctx_set_damping(trpo_ctx *c, double d) {
    if (!c) return TRPO_E_INVALID;
    c->damping = d;
    if (c->twin) trpo_dev_set_damping(c->twin, d);
    return trpo_dev_set_damping(c->dev, d);
}
size_t trpo_ctx_num_params(const trpo_ctx *c) { return c ? c->P : 0; }

int trpo_comm_unique_id(void *id) {
    if (!id) return TRPO_E_INVALID;
    return trpo_dev_comm_unique_id(id);
}
int trpo_ctx_attach_comm(trpo_ctx *c, int rank, int world, const void *id) {
    return trpo_ctx_attach_comm_timeout(c, rank, world, id, 0);
}
int trpo_ctx_attach_comm_timeout(trpo_ctx *c, int rank, int world, const void *id, long timeout_ms) {
    if (!c || (world > 1 && !id)) return TRPO_E_INVALID;
    drop_twin(c);
    const int rc = trpo_dev_set_comm(c->dev, rank, world, id, timeout_ms);
    if (rc == TRPO_E_TIMEOUT) set_err("RCCL init (rank %d of %d) did not complete within its time limit", rank, world);
    else if (rc) set_err("RCCL attach (rank %d of %d) failed (code %d; ncclCommInitRank's reason on stderr)", rank, world, rc);
    return rc;
}
int trpo_ctx_comm_verify(trpo_ctx *c, long timeout_ms) {
    if (!c) return TRPO_E_INVALID;
    long bad = 0;
    const int rc = trpo_dev_comm_verify(c->dev, timeout_ms, &bad);
    if (rc == TRPO_E_VERIFY) set_err("collective self-check: %ld elements of the test all-reduce differ from the exact sum", bad);
    else if (rc == TRPO_E_TIMEOUT) set_err("collective self-check: the test all-reduce did not complete in time");
    return rc;
}
int trpo_ctx_wait(trpo_ctx *c, long timeout_ms) {
    if (!c) return TRPO_E_INVALID;
    const int rc = trpo_dev_wait(c->dev, timeout_ms);
    if (rc == TRPO_E_TIMEOUT) set_err("the context's stream did not complete in time");
    return rc;
}
int trpo_ctx_comm_abort(trpo_ctx *c) { return c ? trpo_dev_comm_abort(c->dev) : TRPO_E_INVALID; }

trpo_group *trpo_group_create(int world) { return (trpo_group *)trpo_hgroup_create(world); }
void trpo_group_destroy(trpo_group *g) { trpo_hgroup_destroy((trpo_hgroup *)g); }
int trpo_ctx_attach_group(trpo_ctx *c, trpo_group *g, int rank) {
    if (!c || !g) return TRPO_E_INVALID;
    const int rc = trpo_dev_set_group(c->dev, (trpo_hgroup *)g, rank);
    if (rc) set_err("attach_group(rank %d) failed (code %d)", rank, rc);
    return rc;
}
int trpo_ctx_comm_info(const trpo_ctx *c, int *rank, int *world, int *replicas) {
    return c ? trpo_dev_comm_info(c->dev, rank, world, replicas) : TRPO_E_INVALID;
}

int trpo_ctx_peer_handle(trpo_ctx *c, void *handle_64) {
    if (!c) return TRPO_E_INVALID;
    const int rc = trpo_dev_peer_open(c->dev, handle_64);
    if (rc) set_err("peer window open / IPC export failed (code %d)", rc);
    return rc;
}
int trpo_ctx_attach_peers(trpo_ctx *c, int rank, int world, const void *handles) {
    if (!c || !handles) return TRPO_E_INVALID;
    int rc = trpo_dev_peer_open(c->dev, NULL);
    if (!rc) rc = trpo_dev_set_peers(c->dev, rank, world, handles, NULL);
    if (rc) set_err("attach_peers(rank %d of %d) failed (code %d)", rank, world, rc);
    return rc;
}
int trpo_ctx_attach_peers_local(trpo_ctx *c, int rank, int world, trpo_ctx *const *all) {
    if (!c || !all || world < 1 || world > TRPO_PEER_MAX_RANKS) return TRPO_E_INVALID;
    void *w[TRPO_PEER_MAX_RANKS];
    for (int r = 0; r < world; ++r) {
        w[r] = all[r] ? trpo_dev_peer_window(all[r]->dev) : NULL;
        if (!w[r]) {
            set_err("attach_peers_local: rank %d has no open peer window (trpo_ctx_peer_handle first)", r);
            return TRPO_E_INVALID;
        }
    }
    const int rc = trpo_dev_set_peers(c->dev, rank, world, NULL, w);
    if (rc) set_err("attach_peers_local(rank %d of %d) failed (code %d)", rank, world, rc);
    return rc;
}
const char *trpo_ctx_comm_backend(const trpo_ctx *c) { return c ? trpo_dev_comm_backend(c->dev) : ""; }

int trpo_ctx_surrogate(trpo_ctx *c, const double *fullstep, int k0, int nk, double *surr) {
    if (!c || !fullstep || !surr || k0 < 0 || nk < 1 || nk > 64) return TRPO_E_INVALID;
    if (!c->have_roll) {
        set_err("surrogate: no rollout uploaded for the current samples (trpo_ctx_set_rollout)");
        return TRPO_E_INVALID;
    }
    const int rc = trpo_dev_surrogate(c->dev, fullstep, k0, nk, surr);
    if (rc) set_err("surrogate failed on the device (code %d)", rc);
    return rc;
}

double trpo_ctx_fvp(trpo_ctx *c, const double *v, double *out) {
    if (!c || !v || !out) return TRPO_E_INVALID;
    const double t0 = now_s();
    int rc = trpo_dev_upload(c->dev, TRPO_VEC_V, v);
    if (!rc) rc = trpo_dev_fvp_host(c->dev, out);
    if (rc) {
        set_err("FVP failed on the device (code %d)", rc);
        return rc < 0 ? rc : TRPO_E_DEVICE;
    }
    return now_s() - t0;
}

double trpo_ctx_cg(trpo_ctx *c, const double *b, size_t max_iter, double th, double *x, int verbose) {
    if (!c || !b || !x) return TRPO_E_INVALID;
    const double t0 = now_s();
    double stats[TRPO_CG_STATS], rdh[66];
    size_t its = 0;
    trpo_dev *hd = c->dev;                             /* the context whose solve x comes from */
    c->last_rerun = 0;
    int rc = trpo_dev_upload(c->dev, TRPO_VEC_B, b);
    if (!rc) rc = trpo_dev_cg(c->dev, max_iter, th);
    if (!rc) rc = trpo_dev_download_x_cg(c->dev, x, stats, rdh, 66, &its);
    if (!rc && needs_rerun(c, stats, rdh, its)) {
        trpo_dev *t = get_twin(c);
        if (t) {
            rc = trpo_dev_upload(t, TRPO_VEC_B, b);
            if (!rc) rc = trpo_dev_cg(t, max_iter, th);
            if (!rc) rc = trpo_dev_download(t, TRPO_VEC_X, x);
            /* the context's own slot X then holds the x this call returns (trpo_ctx_download_x agrees) */
            if (!rc) rc = trpo_dev_upload(c->dev, TRPO_VEC_X, x);
            if (!rc) {
                c->last_rerun = 1;
                hd = t;
                fprintf(stderr, "[WARN] CG: a Ritz value converged to %.1e (relative residual), where the "
                                "reference's fp64 CG loses orthogonality; solved again in fp64\n", c->last_ritz);
            }
        } else {
            fprintf(stderr, "[WARN] CG: a Ritz value converged to %.1e and the fp64 re-solve is unavailable: %s\n",
                    c->last_ritz, g_err);
        }
    }
    const double t1 = now_s();
    if (rc) {
        set_err("CG failed on the device (code %d)", rc);
        return rc < 0 ? rc : TRPO_E_DEVICE;
    }
    if (verbose) {
        /* src/TRPO_CG.c:56 -- one line per iteration, rdotr is the squared norm */
        size_t iters = 0;
        double *rr = (double *)malloc(sizeof(double) * (max_iter + 1));
        double *xn = (double *)malloc(sizeof(double) * (max_iter + 1));
        if (rr && xn && !trpo_dev_cg_history(hd, rr, xn, max_iter + 1, &iters)) {
            for (size_t i = 0; i <= iters; ++i)
                printf("CG Iter[%zu] Residual Norm=%.12e, Soln Norm=%.12e\n", i, rr[i], xn[i]);
        }
        free(rr);
        free(xn);
    }
    return t1 - t0;
}

int trpo_ctx_cg_history(const trpo_ctx *c, double *rdotr, double *xnorm, size_t cap, size_t *iters) {
    if (!c) return TRPO_E_INVALID;
    return trpo_dev_cg_history(c->last_rerun && c->twin ? c->twin : c->dev, rdotr, xnorm, cap, iters);
}

int trpo_ctx_cg_status(const trpo_ctx *c, double *ritz_residual, double *orth_loss, int *fp64_rerun) {
    if (!c) return TRPO_E_INVALID;
    if (ritz_residual) *ritz_residual = c->last_ritz;
    if (orth_loss) *orth_loss = c->last_orth;
    if (fp64_rerun) *fp64_rerun = c->last_rerun;
    return 0;
}

/* ------------------------------------------------------------------------- */
/* one TRPO policy update (src/TRPO_Update.c:254-1007)                       */
/* ------------------------------------------------------------------------- */
int trpo_ctx_set_rollout(trpo_ctx *c, const double *mean, const double *action, const double *adv) {
    if (!c || (c->n && (!mean || !action || !adv))) return TRPO_E_INVALID;
    drop_twin(c);
    int rc = trpo_dev_set_rollout(c->dev, mean, action, adv, c->n);
    c->have_roll = rc == 0;
    if (rc) set_err("rollout upload failed (code %d)", rc);
    return rc;
}

double trpo_ctx_update(trpo_ctx *c, size_t max_iter, double resth, double max_kl, int max_bt, double accept,
                       double *theta_out, double *b_out, double *x_out, trpo_update_info *info, int verbose) {
    if (!c || !theta_out || max_bt < 0 || max_bt > TRPO_MAX_BACKTRACKS || !(max_kl > 0)) return TRPO_E_INVALID;
    if (!c->have_roll) {
        set_err("trpo_ctx_update: no rollout for the current samples (trpo_ctx_set_rollout)");
        return TRPO_E_INVALID;
    }
    const size_t P = c->P;
    double *b = (double *)malloc(sizeof(double) * P), *x = (double *)malloc(sizeof(double) * P);
    double *z = (double *)malloc(sizeof(double) * P), *fullstep = (double *)malloc(sizeof(double) * P);
    trpo_update_info inf;
    memset(&inf, 0, sizeof inf);
    inf.accepted = -1;
    double ret = TRPO_E_NOMEM;
    if (!b || !x || !z || !fullstep) goto out;
    const double t0 = now_s();
    double adv_sum = 0.0, surr0 = 0.0, shs_lm[2] = {0.0, 0.0};
    /* policy gradient (:254-378), CG (:383-628) and FVP(x) (:633-832) on the device, one sync */
    double *rr = (double *)malloc(sizeof(double) * (max_iter + 1));
    double *xn = (double *)malloc(sizeof(double) * (max_iter + 1));
    double stats[TRPO_CG_STATS];
    trpo_dev *dv = c->dev;                 /* the context the update's results come from */
    c->last_rerun = 0;
    int rc = (!rr || !xn) ? TRPO_E_NOMEM
                          : trpo_dev_update_solve(c->dev, max_iter, resth, b, x, z, &adv_sum, &inf.cg_iters, rr, xn,
                                                  max_kl, max_bt > 0 ? &surr0 : NULL, shs_lm, stats);
    if (!rc && needs_rerun(c, stats, rr, inf.cg_iters < max_iter ? inf.cg_iters : max_iter)) {
        /* the fp32 stall guard: the whole device phase again on the fp64 twin (its line search too) */
        trpo_dev *t = get_twin(c);
        if (t) {
            rc = trpo_dev_update_solve(t, max_iter, resth, b, x, z, &adv_sum, &inf.cg_iters, rr, xn, max_kl,
                                       max_bt > 0 ? &surr0 : NULL, shs_lm, NULL);
            if (!rc) {
                dv = t;
                c->last_rerun = 1;
                fprintf(stderr, "[WARN] TRPO_Update: a Ritz value of the CG solve converged to %.1e (relative "
                                "residual), where the reference's fp64 CG loses orthogonality; update solved again "
                                "in fp64\n", c->last_ritz);
            }
        } else {
            fprintf(stderr, "[WARN] TRPO_Update: a Ritz value converged to %.1e and the fp64 re-solve is "
                            "unavailable: %s\n", c->last_ritz, g_err);
        }
    }
    if (!rc && verbose) /* src/TRPO_CG.c:56 -- one line per iteration */
        for (size_t i = 0; i <= inf.cg_iters && i <= max_iter; ++i)
            printf("CG Iter[%zu] Residual Norm=%.12e, Soln Norm=%.12e\n", i, rr[i], xn[i]);
    free(rr);
    free(xn);
    if (rc) {
        set_err("TRPO update failed on the device (code %d)", rc);
        ret = rc < 0 ? rc : TRPO_E_DEVICE;
        goto out;
    }
    /* step size (src/TRPO_Update.c:834-868), fp64 on the host, reference order */
    /* shs = 0.5 x.Fx and lm = sqrt(shs / max_kl) (:836-846) as the device summed them: its fullstep
     * x / lm -- the first line-search candidate it already evaluated -- is the one below, bit for bit */
    const double shs = shs_lm[0];
    if (verbose) printf("shs: %.14f\n", shs);
    const double lm = shs_lm[1];
    double gnorm = 0;
    for (size_t i = 0; i < P; ++i) gnorm += b[i] * b[i];
    gnorm = sqrt(gnorm);
    if (verbose) printf("lagrange multiplier: %.14f, gnorm: %.14f\n", lm, gnorm);
    for (size_t i = 0; i < P; ++i) fullstep[i] = x[i] / lm;
    double neggdotstepdir = 0;
    for (size_t i = 0; i < P; ++i) neggdotstepdir += b[i] * x[i];
    memcpy(theta_out, x, P * sizeof(double));        /* reference quirk: theta starts as x */
    const double rate = neggdotstepdir / lm;
    const double N = trpo_dev_n_total(dv);
    const double fval = -adv_sum / N;
    if (verbose) printf("fval before %.14e\n", fval);
    inf.shs = shs;
    inf.lagrange = lm;
    inf.gnorm = gnorm;
    inf.fval_before = fval;
    inf.expected_improve_rate = rate;
    /* backtracking line search (src/TRPO_Update.c:884-1007): fraction 1 alone first
     * (the usual outcome), then every remaining fraction in one launch; the accepted
     * one is the first in order, exactly as the sequential reference loop finds it */
    for (int k0 = 0; k0 < max_bt && inf.accepted < 0;) {
        const int nk = k0 == 0 ? 1 : max_bt - k0;
        double surr[TRPO_MAX_BACKTRACKS];
        if (k0 == 0)
            surr[0] = surr0;       /* evaluated by the device with the solve (same fullstep, bit for bit) */
        else
            rc = trpo_dev_surrogate(dv, fullstep, k0, nk, surr);
        if (rc) {
            set_err("line search failed on the device (code %d)", rc);
            ret = rc < 0 ? rc : TRPO_E_DEVICE;
            goto out;
        }
        for (int j = 0; j < nk; ++j) {
            const int k = k0 + j;
            const double stepfrac = pow(0.5, (double)k);
            const double newfval = -surr[j] / N;
            const double actual = fval - newfval, expected = rate * stepfrac, ratio = actual / expected;
            if (verbose) printf("a/e/r %.14f / %.14f / %.14f\n", actual, expected, ratio);
            inf.actual[k] = actual;
            inf.expected[k] = expected;
            inf.ratio[k] = ratio;
            inf.evaluated = k + 1;
            if (ratio > accept && actual > 0) {
                for (size_t i = 0; i < P; ++i) theta_out[i] = c->theta[i] + stepfrac * fullstep[i];
                inf.accepted = k;
                break;
            }
        }
        k0 += nk;
    }
    ret = now_s() - t0;
    if (b_out) memcpy(b_out, b, P * sizeof(double));
    if (x_out) memcpy(x_out, x, P * sizeof(double));
    if (info) *info = inf;
out:
    free(b);
    free(x);
    free(z);
    free(fullstep);
    return ret;
}

int trpo_ctx_upload_b(trpo_ctx *c, const double *b) { return c ? trpo_dev_upload(c->dev, TRPO_VEC_B, b) : -1; }
int trpo_ctx_upload_v(trpo_ctx *c, const double *v) { return c ? trpo_dev_upload(c->dev, TRPO_VEC_V, v) : -1; }
int trpo_ctx_enqueue_fvp(trpo_ctx *c) { return c ? trpo_dev_fvp(c->dev) : -1; }
int trpo_ctx_enqueue_cg(trpo_ctx *c, size_t m, double th) { return c ? trpo_dev_cg(c->dev, m, th) : -1; }
int trpo_ctx_enqueue_fvp_kernel_only(trpo_ctx *c) { return c ? trpo_dev_fvp_kernel(c->dev) : -1; }
int trpo_ctx_synchronize(trpo_ctx *c) { return c ? trpo_dev_sync(c->dev) : -1; }
double trpo_ctx_time(trpo_ctx *c, int what, int reps, size_t m, double th) {
    return c ? trpo_dev_time(c->dev, what, reps, m, th) : -1;
}
int trpo_ctx_download_x(trpo_ctx *c, double *x) { return c ? trpo_dev_download(c->dev, TRPO_VEC_X, x) : -1; }
int trpo_ctx_download_z(trpo_ctx *c, double *z) { return c ? trpo_dev_download(c->dev, TRPO_VEC_Z, z) : -1; }
const char *trpo_ctx_kernel_name(const trpo_ctx *c) { return c ? trpo_dev_kernel_name(c->dev) : ""; }
int trpo_ctx_launch_geometry(const trpo_ctx *c, int *b, int *t, int *l) {
    return c ? trpo_dev_geometry(c->dev, b, t, l) : -1;
}

/* ------------------------------------------------------------------------- */
/* reference text formats                                                    */
/* ------------------------------------------------------------------------- */
/* slurp / load_model / load_data live in trpo_textio.c (a CPU-only unit, also built under
 * AddressSanitizer + UBSan by `make -C oracle asan`) */
#define load_model trpo_text_load_model
#define load_data trpo_text_load_data

/* Optional forward-pass check of the data file's Mean column (src/TRPO_FVP.c:839-844),
 * enabled with TRPO_CHECK_MEAN=1; done once when a data file is (re)loaded. */
static void check_mean(const trpo_ctx *c, const double *theta, const double *obs, const double *mean, size_t n) {
    size_t maxw = 0;
    for (size_t i = 0; i < c->nl; ++i) maxw = c->ls[i] > maxw ? c->ls[i] : maxw;
    double *a = (double *)malloc(maxw * sizeof(double)), *b = (double *)malloc(maxw * sizeof(double));
    for (size_t s = 0; s < n; ++s) {
        memcpy(a, obs + s * c->ls[0], c->ls[0] * sizeof(double));
        size_t pos = 0;
        for (size_t i = 0; i + 1 < c->nl; ++i) {
            const size_t in = c->ls[i], out = c->ls[i + 1];
            for (size_t j = 0; j < out; ++j) {
                double x = theta[pos + in * out + j];
                for (size_t k = 0; k < in; ++k) x += a[k] * theta[pos + k * out + j];
                switch (c->ac[i + 1]) {
                case 't': x = tanh(x); break;
                case 'o': x = 0.1 * x; break;
                case 's': x = 1.0 / (1 + exp(-x)); break;
                default: break;
                }
                b[j] = x;
            }
            memcpy(a, b, out * sizeof(double));
            pos += in * out + out;
        }
        const size_t A = c->ls[c->nl - 1];
        for (size_t i = 0; i < A; ++i) {
            const double e = mean[s * A + i], err = fabs((a[i] - e) / e) * 100;
            if (err > 1) printf("out[%zu] = %e, mean = %e => %.4f%% Difference\n", i, a[i], e, err);
        }
    }
    free(a);
    free(b);
}

/* ------------------------------------------------------------------------- */
/* file-keyed cache for the TRPOparam entry points                           */
/* ------------------------------------------------------------------------- */
#define CACHE_SLOTS 4

typedef struct {
    int used;
    unsigned long long stamp;
    char *model, *data;
    off_t msize, dsize;
    struct timespec mmtime, dmtime;
    size_t nsamples, nl, ls[MAX_LAYERS];
    char ac[MAX_LAYERS + 1];
    trpo_ctx *ctx;
    int has_roll;              /* Mean/Action/Adv uploaded (TRPO_Update) */
} cache_entry;

static cache_entry g_cache[CACHE_SLOTS];
static unsigned long long g_clock;
static pthread_mutex_t g_lock = PTHREAD_MUTEX_INITIALIZER;

static void entry_free(cache_entry *e) {
    if (!e->used) return;
    trpo_ctx_destroy(e->ctx);
    free(e->model);
    free(e->data);
    memset(e, 0, sizeof *e);
}

void trpo_cache_clear(void) {
    pthread_mutex_lock(&g_lock);
    for (int i = 0; i < CACHE_SLOTS; ++i) entry_free(&g_cache[i]);
    pthread_mutex_unlock(&g_lock);
}

static int same_ts(struct timespec a, struct timespec b) { return a.tv_sec == b.tv_sec && a.tv_nsec == b.tv_nsec; }

/* Upload Mean/Action/Adv of the data file into a cached context (TRPO_Update). */
static int load_rollout(cache_entry *e, const TRPOparam *prm) {
    const size_t nl = prm->NumLayers, O = prm->LayerSize[0], A = prm->LayerSize[nl - 1], n = prm->NumSamples;
    double *obs = (double *)calloc(n * O + 1, sizeof(double)), *stdv = (double *)calloc(A, sizeof(double));
    double *mean = (double *)calloc(n * A + 1, sizeof(double)), *act = (double *)calloc(n * A + 1, sizeof(double));
    double *adv = (double *)calloc(n + 1, sizeof(double));
    int rc = -1;
    if (obs && stdv && mean && act && adv && !load_data(prm->DataFile, O, A, n, obs, stdv, mean, act, adv))
        rc = trpo_ctx_set_rollout(e->ctx, mean, act, adv);
    if (!rc) e->has_roll = 1;
    free(obs);
    free(stdv);
    free(mean);
    free(act);
    free(adv);
    return rc;
}

/* Returns a context for param (parsing + uploading on a miss), or NULL with the
 * reference's "[ERROR] Cannot open ..." message on stderr.  need_roll: also make
 * sure the rollout columns are on the device (TRPO_Update). */
static trpo_ctx *ctx_for_param(const TRPOparam *prm, int need_roll) {
    if (!prm->ModelFile || !prm->DataFile) {
        fprintf(stderr, "[ERROR] Model/Data file name missing.\n");
        return NULL;
    }
    if (check_shape(prm->NumLayers, prm->LayerSize, prm->AcFunc)) {
        fprintf(stderr, "[ERROR] %s\n", g_err);
        return NULL;
    }
    struct stat sm, sd;
    if (stat(prm->ModelFile, &sm) != 0) {
        fprintf(stderr, "[ERROR] Cannot open Model File [%s]. \n", prm->ModelFile);
        return NULL;
    }
    if (stat(prm->DataFile, &sd) != 0) {
        fprintf(stderr, "[ERROR] Cannot open Data File [%s]. \n", prm->DataFile);
        return NULL;
    }
    cache_entry *hit = NULL, *victim = &g_cache[0];
    for (int i = 0; i < CACHE_SLOTS; ++i) {
        cache_entry *e = &g_cache[i];
        if (!e->used) {
            if (victim->used) victim = e;
            continue;
        }
        if (victim->used && e->stamp < victim->stamp) victim = e;
        if (strcmp(e->model, prm->ModelFile) || strcmp(e->data, prm->DataFile)) continue;
        if (e->msize != sm.st_size || e->dsize != sd.st_size || !same_ts(e->mmtime, sm.st_mtim) ||
            !same_ts(e->dmtime, sd.st_mtim))
            continue;
        if (e->nsamples != prm->NumSamples || e->nl != prm->NumLayers) continue;
        if (memcmp(e->ls, prm->LayerSize, prm->NumLayers * sizeof(size_t)) ||
            memcmp(e->ac, prm->AcFunc, prm->NumLayers))
            continue;
        hit = e;
        break;
    }
    if (hit) {
        hit->stamp = ++g_clock;
        if (need_roll && !hit->has_roll && load_rollout(hit, prm)) return NULL;
        return hit->ctx;
    }
    /* miss: parse both files, upload, replace the LRU slot */
    const size_t nl = prm->NumLayers, O = prm->LayerSize[0], A = prm->LayerSize[nl - 1], n = prm->NumSamples;
    const size_t P = NumParamsCalc(prm->LayerSize, nl);
    double *theta = (double *)calloc(P, sizeof(double));
    double *obs = (double *)calloc(n * O + 1, sizeof(double));
    double *stdv = (double *)calloc(A, sizeof(double));
    const char *cm = getenv("TRPO_CHECK_MEAN");
    const int want_mean = cm && atoi(cm);
    double *mean = want_mean ? (double *)calloc(n * A + 1, sizeof(double)) : NULL;
    trpo_ctx *ctx = NULL;
    if (!theta || !obs || !stdv) goto out;
    if (load_model(prm->ModelFile, P, theta)) goto out;
    /* FVPFast reads "LogStd" from the model into Std; the data file overwrites it */
    for (size_t k = 0; k < A; ++k) stdv[k] = theta[P - A + k];
    if (load_data(prm->DataFile, O, A, n, obs, stdv, mean, NULL, NULL)) goto out;
    ctx = trpo_ctx_create(nl, prm->LayerSize, prm->AcFunc, theta, obs, n, stdv, prm->CG_Damping, -1);
    if (!ctx) {
        fprintf(stderr, "[ERROR] %s\n", g_err);
        goto out;
    }
    if (want_mean) check_mean(ctx, theta, obs, mean, n);
    entry_free(victim);
    victim->used = 1;
    victim->stamp = ++g_clock;
    victim->model = strdup(prm->ModelFile);
    victim->data = strdup(prm->DataFile);
    victim->msize = sm.st_size;
    victim->dsize = sd.st_size;
    victim->mmtime = sm.st_mtim;
    victim->dmtime = sd.st_mtim;
    victim->nsamples = n;
    victim->nl = nl;
    memcpy(victim->ls, prm->LayerSize, nl * sizeof(size_t));
    memset(victim->ac, 0, sizeof victim->ac);
    memcpy(victim->ac, prm->AcFunc, nl);
    victim->ctx = ctx;
    victim->has_roll = 0;
    if (need_roll && load_rollout(victim, prm)) ctx = NULL;
out:
    free(theta);
    free(obs);
    free(stdv);
    free(mean);
    return ctx;
}

/* ------------------------------------------------------------------------- */
/* the reference entry points                                                */
/* ------------------------------------------------------------------------- */

/* src/TRPO_FVP.c:548-949.  NumThreads sized the reference's OpenMP team; the
 * GPU path has no host compute, so it is accepted and ignored. */
double FVPFast(TRPOparam param, double *Result, double *Input, size_t NumThreads) {
    (void)NumThreads;
    if (!Result || !Input) return -1;
    pthread_mutex_lock(&g_lock);
    trpo_ctx *c = ctx_for_param(&param, 0);
    double t = -1;
    if (c) {
        if (c->damping != param.CG_Damping) trpo_ctx_set_damping(c, param.CG_Damping);
        t = trpo_ctx_fvp(c, Input, Result);
        if (t < 0) {
            fprintf(stderr, "[ERROR] %s\n", g_err);
            t = -1;
        }
    }
    pthread_mutex_unlock(&g_lock);
    return t;
}

/* src/TRPO_FVP.c:11-545: the 4-pass original; mathematically identical to
 * FVPFast because the KL gradient at the old parameters is zero (GLayer=0,
 * src/TRPO_FVP.c:326).  Prints its timing line like the reference (:525). */
double FVP(TRPOparam param, double *Result, double *Input) {
    double t = FVPFast(param, Result, Input, 1);
    if (t >= 0) printf("[INFO] FVP Computing Time is %f seconds.\n", t);
    return t;
}

/* src/TRPO_CG.c:11-113. */
double CG(TRPOparam param, double *Result, double *b, size_t MaxIter, double ResidualTh, size_t NumThreads) {
    (void)NumThreads;
    if (!Result || !b) return -1;
    pthread_mutex_lock(&g_lock);
    trpo_ctx *c = ctx_for_param(&param, 0);
    double t = -1;
    if (c) {
        if (c->damping != param.CG_Damping) trpo_ctx_set_damping(c, param.CG_Damping);
        t = trpo_ctx_cg(c, b, MaxIter, ResidualTh, Result, 1);
        if (t < 0) {
            fprintf(stderr, "[ERROR] Fisher Vector Product Calculation Failed.\n");
            t = -1;
        }
    } else {
        fprintf(stderr, "[ERROR] Fisher Vector Product Calculation Failed.\n");
    }
    fflush(stdout);
    pthread_mutex_unlock(&g_lock);
    return t;
}

/* Accelerator twins (src/include/TRPO.h:98,101): same contract, the MI355X
 * path serves them; PaddedLayerSize / NumBlocks are FPGA-only and ignored. */
double FVP_FPGA(TRPOparam param, double *Result, double *Input) { return FVPFast(param, Result, Input, 1); }

double CG_FPGA(TRPOparam param, double *Result, double *b, size_t MaxIter, double ResidualTh, size_t NumThreads) {
    return CG(param, Result, b, MaxIter, ResidualTh, NumThreads);
}

/* src/TRPO_Update.c:10-1011 with its hard-wired settings: CG MaxIter 10 and
 * ResidualTh 1e-10, MaxKL 0.01, 10 backtracks, AcceptRatio 0.1.  Result receives
 * the updated parameters (or the CG step direction if no backtrack is accepted,
 * like the reference).  The Std of the data file's last line is the FVP sigma;
 * exp(LogStd) of the model is the policy sigma of the gradient and line search. */
double TRPO_Update(TRPOparam param, double *Result, size_t NumThreads) {
    (void)NumThreads;
    if (!Result) return -1;
    pthread_mutex_lock(&g_lock);
    trpo_ctx *c = ctx_for_param(&param, 1);
    double t = -1;
    if (c) {
        if (c->damping != param.CG_Damping) trpo_ctx_set_damping(c, param.CG_Damping);
        t = trpo_ctx_update(c, 10, 1e-10, 0.01, 10, 0.1, Result, NULL, NULL, NULL, 1);
        if (t < 0) {
            fprintf(stderr, "[ERROR] %s\n", g_err);
            t = -1;
        }
    }
    fflush(stdout);
    pthread_mutex_unlock(&g_lock);
    return t;
}

/* ------------------------------------------------------------------------- */
/* value-baseline objective for L-BFGS (src/TRPO_Baseline.c:29-240)          */
/* ------------------------------------------------------------------------- */
struct trpo_baseline {
    trpo_bdev *dev;
    size_t nl, ls[MAX_LAYERS];
    char ac[MAX_LAYERS + 1];
    size_t np;                 /* weights + biases */
    size_t n;
    double *gsum;              /* np + 2 */
    double *obs_h, *tgt_h;     /* last uploaded data (drop-in change detection) */
    size_t cap;
};

trpo_baseline *trpo_baseline_create(size_t num_layers, const size_t *layer_size, const char *acfunc, int device) {
    if (check_shape(num_layers, layer_size, acfunc)) return NULL;
    for (size_t i = 1; i < num_layers; ++i)
        if (acfunc[i] != 'l' && acfunc[i] != 't') {   /* evaluate() knows only these (:120-128) */
            set_err("Activation Function for Layer [%zu] is %c. Unsupported.", i, acfunc[i]);
            return NULL;
        }
    if (layer_size[num_layers - 1] != 1) {
        set_err("the baseline predicts one value (LayerSizeBase[last] = 1)");
        return NULL;
    }
    trpo_baseline *b = (trpo_baseline *)calloc(1, sizeof(trpo_baseline));
    if (!b) return NULL;
    b->nl = num_layers;
    memcpy(b->ls, layer_size, num_layers * sizeof(size_t));
    memcpy(b->ac, acfunc, num_layers);
    b->np = NumParamsCalc(b->ls, b->nl) - 1;
    b->gsum = (double *)calloc(b->np + 2, sizeof(double));
    char err[256] = {0};
    b->dev = trpo_bdev_create(device, num_layers, layer_size, acfunc, err, sizeof err);
    if (!b->dev || !b->gsum) {
        set_err("%s", err[0] ? err : "baseline allocation failed");
        trpo_baseline_destroy(b);
        return NULL;
    }
    return b;
}

void trpo_baseline_destroy(trpo_baseline *b) {
    if (!b) return;
    trpo_bdev_destroy(b->dev);
    free(b->gsum);
    free(b->obs_h);
    free(b->tgt_h);
    free(b);
}

int trpo_baseline_set_data(trpo_baseline *b, const double *observ, const double *target, size_t num_ep,
                           size_t ep_len) {
    if (!b || !observ || !target || !num_ep || !ep_len) return TRPO_E_INVALID;
    const size_t n = num_ep * ep_len, O = b->ls[0] - 1, L0 = b->ls[0];
    double *x = (double *)malloc(sizeof(double) * n * L0);
    if (!x) return TRPO_E_NOMEM;
    for (size_t s = 0; s < n; ++s) {          /* input = [Obs, currentStep / EpLen] (:96-100) */
        memcpy(x + s * L0, observ + s * O, O * sizeof(double));
        x[s * L0 + O] = (double)(s % ep_len) / (double)ep_len;
    }
    int rc = trpo_bdev_set_data(b->dev, x, target, n);
    free(x);
    if (rc) {
        set_err("baseline data upload failed (code %d)", rc);
        return rc < 0 ? rc : TRPO_E_DEVICE;
    }
    b->n = n;
    return 0;
}

/* the objective and gradient from the device's sums in b->gsum */
static double baseline_finish(const trpo_baseline *b, const double *x, double *g, int n) {
    /* gradient (:210-224): sum / N + 0.002 * parameter; zero on the L-BFGS padding */
    const double N = (double)b->n;
    for (size_t q = 0; q < b->np; ++q) g[q] = b->gsum[q] / N + 0.002 * x[q];
    for (int q = (int)b->np; q < n; ++q) g[q] = 0;
    /* objective (:227-240): 0.01 * mean squared error + 0.001 * |x|^2 over the real parameters */
    const double mse = 0.01 * b->gsum[b->np] / N;
    double l2 = 0;
    for (size_t q = 0; q < b->np; ++q) l2 += x[q] * x[q];
    return mse + 0.001 * l2;
}

double trpo_baseline_evaluate(trpo_baseline *b, const double *x, double *g, int n, double *predict) {
    if (!b || !x || !g || n < (int)b->np || !b->n) return TRPO_E_INVALID;
    int rc = trpo_bdev_eval(b->dev, x, b->gsum, predict);
    if (rc) {
        set_err("baseline evaluation failed on the device (code %d)", rc);
        return rc < 0 ? rc : TRPO_E_DEVICE;
    }
    return baseline_finish(b, x, g, n);
}

/* The drop-in for src/TRPO_Baseline.c:29 (liblbfgs callback).  One cached device context per
 * network shape; the sample data is re-uploaded only when its contents change (compared with
 * the last upload), so the ~25 callbacks of one lbfgs() fit upload once. */
static trpo_baseline *g_base;

double evaluate(void *instance, const double *x, double *g, const int n, const double step) {
    (void)step;
    TRPOBaselineParam *p = (TRPOBaselineParam *)instance;
    if (!p || !x || !g || !p->LayerSizeBase || !p->AcFunc || !p->Observ || !p->Target) return -1;
    if (p->NumLayers < 2 || p->LayerSizeBase[0] != p->ObservSpaceDim + 1 ||
        p->NumSamples != p->NumEpBatch * p->EpLen) {
        fprintf(stderr, "[ERROR] inconsistent TRPOBaselineParam (LayerSizeBase[0] = ObservSpaceDim + 1, "
                        "NumSamples = NumEpBatch * EpLen)\n");
        return -1;
    }
    for (size_t i = 1; i < p->NumLayers; ++i)
        if (p->AcFunc[i] != 'l' && p->AcFunc[i] != 't') {
            printf("[ERROR] Activation Function for Layer [%zu] is %c. Unsupported.\n", i, p->AcFunc[i]);
            return -1;
        }
    pthread_mutex_lock(&g_lock);
    double f = -1;
    trpo_baseline *b = g_base;
    if (b && (b->nl != p->NumLayers || memcmp(b->ls, p->LayerSizeBase, p->NumLayers * sizeof(size_t)) ||
              memcmp(b->ac, p->AcFunc, p->NumLayers))) {
        trpo_baseline_destroy(b);
        b = g_base = NULL;
    }
    if (!b) b = g_base = trpo_baseline_create(p->NumLayers, p->LayerSizeBase, p->AcFunc, -1);
    if (b) {
        const size_t N = p->NumSamples, O = p->ObservSpaceDim;
        int rc = 0;
        /* with data already uploaded for this N, the device evaluates on it while the host compares the
         * caller's arrays with that upload (the comparison, ~5 us at 20 x 150, leaves the critical path);
         * if they differ, that result is dropped and the evaluation runs again on the new data */
        const int have = b->n == N && b->cap >= N && b->obs_h && n >= (int)b->np;
        const int started = have && trpo_bdev_eval_start(b->dev, x, p->Predict != NULL) == 0;
        const int same = have && !memcmp(b->obs_h, p->Observ, N * O * sizeof(double)) &&
                         !memcmp(b->tgt_h, p->Target, N * sizeof(double));
        if (started) {
            rc = trpo_bdev_eval_finish(b->dev, b->gsum, p->Predict);
            if (rc) set_err("baseline evaluation failed on the device (code %d)", rc);
            else if (same) f = baseline_finish(b, x, g, n);
        } else if (same) {
            f = trpo_baseline_evaluate(b, x, g, n, p->Predict);   /* the start was refused: its error */
        }
        if (!same && !rc) {
            rc = trpo_baseline_set_data(b, p->Observ, p->Target, p->NumEpBatch, p->EpLen);
            if (!rc && N > b->cap) {
                free(b->obs_h);
                free(b->tgt_h);
                b->obs_h = (double *)malloc(sizeof(double) * N * O + 1);
                b->tgt_h = (double *)malloc(sizeof(double) * N + 1);
                b->cap = (b->obs_h && b->tgt_h) ? N : 0;
            }
            if (!rc && b->cap >= N) {
                memcpy(b->obs_h, p->Observ, N * O * sizeof(double));
                memcpy(b->tgt_h, p->Target, N * sizeof(double));
            }
            if (!rc) f = trpo_baseline_evaluate(b, x, g, n, p->Predict);
        }
        /* the reference leaves W/B = x in the param's arrays (:64-81) */
        if (f >= 0 && p->WBase && p->BBase) {
            size_t pos = 0;
            for (size_t i = 0; i + 1 < p->NumLayers; ++i) {
                const size_t cur = p->LayerSizeBase[i], nxt = p->LayerSizeBase[i + 1];
                if (p->WBase[i]) memcpy(p->WBase[i], x + pos, cur * nxt * sizeof(double));
                pos += cur * nxt;
                if (p->BBase[i]) memcpy(p->BBase[i], x + pos, nxt * sizeof(double));
                pos += nxt;
            }
        }
        if (f < 0) fprintf(stderr, "[ERROR] %s\n", g_err);
    } else {
        fprintf(stderr, "[ERROR] %s\n", g_err);
    }
    pthread_mutex_unlock(&g_lock);
    return f;
}
