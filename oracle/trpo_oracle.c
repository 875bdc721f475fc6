/*
 * trpo_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Clean-room CPU restatement (IEEE fp64) of the reference TRPO Fisher-vector
 * product and conjugate-gradient solve.  It is the *checker* for the MI355X
 * path and the "port" CPU baseline timed by bench.py; nothing in the product
 * library (trpo-robot-control_amd/) links, loads or calls it.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.
 *
 * Parity is PINNED: tests/test_oracle.py checks this file against goldens
 * produced by the reference's own TRPO_FVP.c / TRPO_CG.c compiled unchanged
 * (oracle/Makefile -> oracle/_ref/, driver oracle/ref_driver.c) and against
 * the reference fixture build/ArmTestCG.txt.
 *
 * Reference behaviour restated (paths relative to the reference repo):
 *   - parameter layout  W[i] row-major [in][out], B[i], ..., LogStd[A]
 *                                          src/TRPO_FVP.c:670-699, 704-725
 *   - data-file layout  Mean[A] Std[A] Obs[O] Action[A] Adv per sample;
 *     only Obs and the LAST line's Std are used by the FVP
 *                                          src/TRPO_FVP.c:731-762
 *   - combined forward (y, R{x}, R{y})     src/TRPO_FVP.c:776-836
 *   - Pearlmutter backward (R{g})          src/TRPO_FVP.c:852-900
 *   - sequential accumulation + 2*v_logstd src/TRPO_FVP.c:903-921
 *   - epilogue  Fv = acc/N + damping*v     src/TRPO_FVP.c:928-931
 *   - CG loop, test at the top, <= MaxIter FVPs, prints rdotr/|x|
 *                                          src/TRPO_CG.c:11-113
 *   - NumParamsCalc                        src/TRPO_Util.c:7-17
 *   - TRPO_Update: policy gradient         src/TRPO_Update.c:254-378
 *                  CG (inlined copy)       src/TRPO_Update.c:383-628
 *                  FVP(x), shs, lagrange   src/TRPO_Update.c:633-866
 *                  line search             src/TRPO_Update.c:868-1007
 *                  (theta starts as the CG step x: :850-852 quirk kept)
 *   - value-baseline objective evaluate()  src/TRPO_Baseline.c:29-240
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define OR_MAX_LAYERS 16

static double or_now(void) {
    struct timeval tv;
    gettimeofday(&tv, NULL);
    return (double)tv.tv_sec + 1e-6 * (double)tv.tv_usec;
}

/* src/TRPO_Util.c:7-17 */
size_t oracle_num_params(const size_t *ls, size_t nl) {
    size_t p = 0;
    for (size_t i = 0; i + 1 < nl; ++i) p += ls[i] * ls[i + 1] + ls[i + 1];
    return p + ls[nl - 1];
}

static int or_valid_act(char c) { return c == 'l' || c == 't' || c == 'o' || c == 's'; }

/* One sample of FVPFast's per-sample body (src/TRPO_FVP.c:776-921), adding the
 * sample's contribution into acc[P].  Work arrays are caller-provided. */
typedef struct {
    double *y[OR_MAX_LAYERS], *rx[OR_MAX_LAYERS], *ry[OR_MAX_LAYERS], *rg[OR_MAX_LAYERS];
} or_work;

static void or_sample(size_t nl, const size_t *ls, const char *ac, double *const *W, double *const *B,
                      double *const *VW, double *const *VB, const double *vlogstd, const double *x_in,
                      const double *stdv, or_work *w, double *acc) {
    const size_t A = ls[nl - 1];
    for (size_t i = 0; i < ls[0]; ++i) {
        w->y[0][i] = x_in[i];
        w->rx[0][i] = 0;
        w->ry[0][i] = 0;
    }
    /* combined forward: src/TRPO_FVP.c:783-836 */
    for (size_t i = 0; i + 1 < nl; ++i) {
        const size_t in = ls[i], out = ls[i + 1];
        for (size_t j = 0; j < out; ++j) {
            double xj = B[i][j];
            double rxj = VB[i][j];
            for (size_t k = 0; k < in; ++k) {
                xj += w->y[i][k] * W[i][k * out + j];
                rxj += w->ry[i][k] * W[i][k * out + j];
                rxj += w->y[i][k] * VW[i][k * out + j];
            }
            double yj = xj, ryj = rxj;
            switch (ac[i + 1]) {
            case 'l': ryj = rxj; break;
            case 't': yj = tanh(xj); ryj = rxj * (1 - yj * yj); break;
            case 'o': yj = 0.1 * xj; ryj = 0.1 * rxj; break;
            case 's': yj = 1.0 / (1 + exp(-xj)); ryj = rxj * yj * (1 - yj); break;
            default: break;
            }
            w->y[i + 1][j] = yj;
            w->rx[i + 1][j] = rxj;
            w->ry[i + 1][j] = ryj;
        }
    }
    /* R{g} at the output: src/TRPO_FVP.c:852-854 */
    for (size_t i = 0; i < A; ++i) w->rg[nl - 1][i] = w->ry[nl - 1][i] / stdv[i] / stdv[i];

    /* backward, deepest layer first: src/TRPO_FVP.c:857-900.  Gradients are
     * added straight into acc at their flat positions, in the same per-sample
     * order the reference accumulates them (src/TRPO_FVP.c:903-921). */
    size_t off[OR_MAX_LAYERS];
    {
        size_t pos = 0;
        for (size_t i = 0; i + 1 < nl; ++i) {
            off[i] = pos;
            pos += ls[i] * ls[i + 1] + ls[i + 1];
        }
        off[nl - 1] = pos;
    }
    for (size_t i = nl - 1; i > 0; --i) {
        const size_t cur = ls[i], prev = ls[i - 1];
        double *rg = w->rg[i];
        const double *y = w->y[i];
        for (size_t j = 0; j < cur; ++j) {
            switch (ac[i]) {
            case 't': rg[j] = (1 - y[j] * y[j]) * rg[j]; break;
            case 'o': rg[j] = 0.1 * rg[j]; break;
            case 's': rg[j] = rg[j] * y[j] * (1 - y[j]); break;
            default: break;
            }
        }
        double *aw = acc + off[i - 1];
        double *ab = aw + prev * cur;
        for (size_t j = 0; j < prev; ++j) {
            double t = 0;
            const double yp = w->y[i - 1][j];
            for (size_t k = 0; k < cur; ++k) {
                aw[j * cur + k] += yp * rg[k];
                t += W[i - 1][j * cur + k] * rg[k];
            }
            w->rg[i - 1][j] = t;
        }
        for (size_t k = 0; k < cur; ++k) ab[k] += rg[k];
    }
    for (size_t k = 0; k < A; ++k) acc[off[nl - 1] + k] += 2 * vlogstd[k];
}

/* Fisher-vector product, in memory.  theta: flat parameters (W, B per layer,
 * then LogStd -- the LogStd entries are ignored exactly as FVPFast ignores
 * them).  obs: [n][ls[0]] row-major.  stdv: [A] (the data file's Std).
 * nthreads<=1 reproduces FVPFast's sequential sample order; nthreads>1 splits
 * the samples into contiguous per-thread ranges combined in thread order.
 * Returns compute seconds (FVPFast's timed-region semantics) or -1. */
double oracle_fvp(size_t nl, const size_t *ls, const char *ac, const double *theta, const double *obs,
                  size_t n, const double *stdv, double damping, const double *v, double *out,
                  int nthreads) {
    if (nl < 2 || nl > OR_MAX_LAYERS || n == 0) return -1;
    for (size_t i = 1; i < nl; ++i)
        if (!or_valid_act(ac[i])) {
            fprintf(stderr, "[ERROR] AC Function for Layer[%zu] is %c. Unsupported.\n", i, ac[i]);
            return -1;
        }
    const size_t P = oracle_num_params(ls, nl);
    const size_t A = ls[nl - 1];
    double *W[OR_MAX_LAYERS], *B[OR_MAX_LAYERS], *VW[OR_MAX_LAYERS], *VB[OR_MAX_LAYERS];
    size_t pos = 0;
    for (size_t i = 0; i + 1 < nl; ++i) {
        W[i] = (double *)(theta + pos);
        VW[i] = (double *)(v + pos);
        pos += ls[i] * ls[i + 1];
        B[i] = (double *)(theta + pos);
        VB[i] = (double *)(v + pos);
        pos += ls[i + 1];
    }
    const double *vlogstd = v + pos;
    if (nthreads < 1) nthreads = 1;
    if ((size_t)nthreads > n) nthreads = (int)n;
    size_t maxw = 0;
    for (size_t i = 0; i < nl; ++i) maxw = ls[i] > maxw ? ls[i] : maxw;

    double *accs = (double *)calloc((size_t)nthreads * P, sizeof(double));
    double *work = (double *)calloc((size_t)nthreads * 4 * nl * maxw, sizeof(double));
    if (!accs || !work) {
        free(accs);
        free(work);
        return -1;
    }
    double t0 = or_now();
#ifdef _OPENMP
#pragma omp parallel for num_threads(nthreads) schedule(static, 1)
#endif
    for (int t = 0; t < nthreads; ++t) {
        or_work w;
        double *base = work + (size_t)t * 4 * nl * maxw;
        for (size_t i = 0; i < nl; ++i) {
            w.y[i] = base + (4 * i + 0) * maxw;
            w.rx[i] = base + (4 * i + 1) * maxw;
            w.ry[i] = base + (4 * i + 2) * maxw;
            w.rg[i] = base + (4 * i + 3) * maxw;
        }
        const size_t lo = n * (size_t)t / (size_t)nthreads, hi = n * (size_t)(t + 1) / (size_t)nthreads;
        for (size_t s = lo; s < hi; ++s)
            or_sample(nl, ls, ac, W, B, VW, VB, vlogstd, obs + s * ls[0], stdv, &w, accs + (size_t)t * P);
    }
    for (size_t i = 0; i < P; ++i) {
        double a = accs[i];
        for (int t = 1; t < nthreads; ++t) a += accs[(size_t)t * P + i];
        out[i] = a / (double)n + damping * v[i];
    }
    double t1 = or_now();
    (void)A;
    free(accs);
    free(work);
    return t1 - t0;
}

/* Conjugate gradient (F + damping I) x = b, restating src/TRPO_CG.c:11-113.
 * rdotr_hist / xnorm_hist (length >= maxiter+1, may be NULL) receive the values
 * the reference prints each iteration; *iters gets the number of FVPs done.
 * verbose!=0 prints the reference's per-iteration line.  Returns compute
 * seconds or -1. */
double oracle_cg(size_t nl, const size_t *ls, const char *ac, const double *theta, const double *obs,
                 size_t n, const double *stdv, double damping, const double *b, size_t maxiter,
                 double resth, double *x_out, double *rdotr_hist, double *xnorm_hist, size_t *iters,
                 int nthreads, int verbose) {
    const size_t P = oracle_num_params(ls, nl);
    double *p = (double *)calloc(P, sizeof(double));
    double *r = (double *)calloc(P, sizeof(double));
    double *x = (double *)calloc(P, sizeof(double));
    double *z = (double *)calloc(P, sizeof(double));
    double rdotr = 0, comp = 0;
    size_t nfvp = 0;
    for (size_t i = 0; i < P; ++i) {
        p[i] = b[i];
        r[i] = b[i];
        rdotr += r[i] * r[i];
    }
    for (size_t it = 0; it <= maxiter; ++it) {
        double nrm = 0;
        for (size_t i = 0; i < P; ++i) nrm += x[i] * x[i];
        nrm = sqrt(nrm);
        if (rdotr_hist) rdotr_hist[it] = rdotr;
        if (xnorm_hist) xnorm_hist[it] = nrm;
        if (verbose) printf("CG Iter[%zu] Residual Norm=%.12e, Soln Norm=%.12e\n", it, rdotr, nrm);
        if (rdotr < resth || it == maxiter) {
            memcpy(x_out, x, P * sizeof(double));
            break;
        }
        double ft = oracle_fvp(nl, ls, ac, theta, obs, n, stdv, damping, p, z, nthreads);
        if (ft < 0) {
            free(p); free(r); free(x); free(z);
            return -1;
        }
        comp += ft;
        ++nfvp;
        double t0 = or_now();
        double pz = 0;
        for (size_t i = 0; i < P; ++i) pz += p[i] * z[i];
        const double alpha = rdotr / pz;
        for (size_t i = 0; i < P; ++i) {
            x[i] += alpha * p[i];
            r[i] -= alpha * z[i];
        }
        double nr = 0;
        for (size_t i = 0; i < P; ++i) nr += r[i] * r[i];
        const double beta = nr / rdotr;
        for (size_t i = 0; i < P; ++i) p[i] = r[i] + beta * p[i];
        rdotr = nr;
        comp += or_now() - t0;
    }
    if (iters) *iters = nfvp;
    free(p); free(r); free(x); free(z);
    return comp;
}

/* Model file: one value per line in theta order (src/TRPO_FVP.c:670-699). */
int oracle_load_model(const char *path, size_t nl, const size_t *ls, double *theta) {
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    const size_t P = oracle_num_params(ls, nl);
    for (size_t i = 0; i < P; ++i)
        if (fscanf(f, "%lf", &theta[i]) != 1) {
            fclose(f);
            return -1;
        }
    fclose(f);
    return 0;
}

/* Data file: per sample Mean[A] Std[A] Obs[O] Action[A] Adv
 * (src/TRPO_FVP.c:731-762).  mean may be NULL. */
int oracle_load_data(const char *path, size_t nl, const size_t *ls, size_t n, double *obs, double *stdv,
                     double *mean) {
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    const size_t O = ls[0], A = ls[nl - 1];
    double tmp;
    for (size_t s = 0; s < n; ++s) {
        for (size_t j = 0; j < A; ++j) {
            if (fscanf(f, "%lf", &tmp) != 1) goto bad;
            if (mean) mean[s * A + j] = tmp;
        }
        for (size_t j = 0; j < A; ++j)
            if (fscanf(f, "%lf", &stdv[j]) != 1) goto bad;
        for (size_t j = 0; j < O; ++j)
            if (fscanf(f, "%lf", &obs[s * O + j]) != 1) goto bad;
        for (size_t j = 0; j < A + 1; ++j)
            if (fscanf(f, "%lf", &tmp) != 1) goto bad;
    }
    fclose(f);
    return 0;
bad:
    fclose(f);
    return -1;
}

/* Policy-mean forward pass only (src/TRPO_FVP.c:783-836 without R-ops). */
int oracle_forward(size_t nl, const size_t *ls, const char *ac, const double *theta, const double *obs,
                   size_t n, double *mean_out) {
    size_t maxw = 0;
    for (size_t i = 0; i < nl; ++i) maxw = ls[i] > maxw ? ls[i] : maxw;
    double *a = (double *)malloc(maxw * sizeof(double)), *b = (double *)malloc(maxw * sizeof(double));
    for (size_t s = 0; s < n; ++s) {
        memcpy(a, obs + s * ls[0], ls[0] * sizeof(double));
        size_t pos = 0;
        for (size_t i = 0; i + 1 < nl; ++i) {
            const size_t in = ls[i], out = ls[i + 1];
            const double *Wi = theta + pos, *Bi = theta + pos + in * out;
            for (size_t j = 0; j < out; ++j) {
                double xj = Bi[j];
                for (size_t k = 0; k < in; ++k) xj += a[k] * Wi[k * out + j];
                switch (ac[i + 1]) {
                case 't': xj = tanh(xj); break;
                case 'o': xj = 0.1 * xj; break;
                case 's': xj = 1.0 / (1 + exp(-xj)); break;
                default: break;
                }
                b[j] = xj;
            }
            memcpy(a, b, out * sizeof(double));
            pos += in * out + out;
        }
        memcpy(mean_out + s * ls[nl - 1], a, ls[nl - 1] * sizeof(double));
    }
    free(a);
    free(b);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* TRPO_Update (src/TRPO_Update.c:10-1011)                                   */
/* ------------------------------------------------------------------------- */
static void or_layers(size_t nl, const size_t *ls, const double *theta, const double **W, const double **B,
                      size_t *P) {
    size_t pos = 0;
    for (size_t i = 0; i + 1 < nl; ++i) {
        W[i] = theta + pos;
        pos += ls[i] * ls[i + 1];
        B[i] = theta + pos;
        pos += ls[i + 1];
    }
    *P = pos + ls[nl - 1];
}

/* y[i] = activations of layer i for one sample (src/TRPO_Update.c:262-293) */
static void or_forward1(size_t nl, const size_t *ls, const char *ac, const double *const *W,
                        const double *const *B, const double *x_in, double **y) {
    for (size_t i = 0; i < ls[0]; ++i) y[0][i] = x_in[i];
    for (size_t i = 0; i + 1 < nl; ++i) {
        for (size_t j = 0; j < ls[i + 1]; ++j) {
            double v = B[i][j];
            for (size_t k = 0; k < ls[i]; ++k) v += y[i][k] * W[i][k * ls[i + 1] + j];
            switch (ac[i + 1]) {
            case 't': v = tanh(v); break;
            case 'o': v = 0.1 * v; break;
            case 's': v = 1.0 / (1 + exp(-v)); break;
            default: break;
            }
            y[i + 1][j] = v;
        }
    }
}

/* Policy gradient (src/TRPO_Update.c:254-378).  Rollout: mean/action [n][A], adv [n].
 * normalise != 0 divides by n like the reference; 0 leaves the plain sum (for sharded
 * use).  adv_sum (may be NULL) receives sum(adv) in sample order. */
int oracle_policy_grad(size_t nl, const size_t *ls, const char *ac, const double *theta, const double *obs,
                       const double *mean, const double *action, const double *adv, size_t n, int normalise,
                       double *b, double *adv_sum) {
    if (nl < 2 || nl > OR_MAX_LAYERS) return -1;
    const double *W[OR_MAX_LAYERS], *B[OR_MAX_LAYERS];
    size_t P;
    or_layers(nl, ls, theta, W, B, &P);
    const size_t A = ls[nl - 1];
    const double *logstd = theta + P - A;
    size_t maxw = 0;
    for (size_t i = 0; i < nl; ++i) maxw = ls[i] > maxw ? ls[i] : maxw;
    double *buf = (double *)calloc(2 * nl * maxw + A, sizeof(double));
    double *y[OR_MAX_LAYERS], *g[OR_MAX_LAYERS];
    for (size_t i = 0; i < nl; ++i) {
        y[i] = buf + (2 * i) * maxw;
        g[i] = buf + (2 * i + 1) * maxw;
    }
    double *gls = buf + 2 * nl * maxw;
    memset(b, 0, P * sizeof(double));
    double as = 0;
    for (size_t s = 0; s < n; ++s) {
        or_forward1(nl, ls, ac, W, B, obs + s * ls[0], y);
        for (size_t i = 0; i < A; ++i) {                             /* :297-303 */
            double temp = (action[s * A + i] - mean[s * A + i]) / exp(logstd[i]);
            g[nl - 1][i] = adv[s] * temp / exp(logstd[i]);
            gls[i] = adv[s] * (temp * temp - 1);
        }
        size_t pos = P - A;
        for (size_t i = nl - 1; i > 0; --i) {                        /* :305-357 */
            for (size_t j = 0; j < ls[i]; ++j) {
                switch (ac[i]) {
                case 't': g[i][j] = g[i][j] * (1 - y[i][j] * y[i][j]); break;
                case 'o': g[i][j] = 0.1 * g[i][j]; break;
                case 's': g[i][j] = g[i][j] * y[i][j] * (1 - y[i][j]); break;
                default: break;
                }
            }
            /* accumulate GW[i-1], GB[i-1] at their flat positions (:361-372) */
            pos -= ls[i - 1] * ls[i] + ls[i];
            for (size_t j = 0; j < ls[i - 1]; ++j)
                for (size_t k = 0; k < ls[i]; ++k) b[pos + j * ls[i] + k] += g[i][k] * y[i - 1][j];
            for (size_t k = 0; k < ls[i]; ++k) b[pos + ls[i - 1] * ls[i] + k] += g[i][k];
            for (size_t j = 0; j < ls[i - 1]; ++j) {
                double t = 0;
                for (size_t k = 0; k < ls[i]; ++k) t += g[i][k] * W[i - 1][j * ls[i] + k];
                g[i - 1][j] = t;
            }
        }
        for (size_t k = 0; k < A; ++k) b[P - A + k] += gls[k];
        as += adv[s];
    }
    if (normalise)
        for (size_t i = 0; i < P; ++i) b[i] = b[i] / (double)n;
    if (adv_sum) *adv_sum = as;
    free(buf);
    return 0;
}

/* sum_n Adv_n exp(LLD_n) for parameters theta_new (src/TRPO_Update.c:951-981);
 * stdv = the data file's Std. */
double oracle_surrogate_sum(size_t nl, const size_t *ls, const char *ac, const double *theta_new,
                            const double *obs, const double *mean, const double *action, const double *adv,
                            const double *stdv, size_t n) {
    const double *W[OR_MAX_LAYERS], *B[OR_MAX_LAYERS];
    size_t P;
    or_layers(nl, ls, theta_new, W, B, &P);
    const size_t A = ls[nl - 1];
    const double *logstd = theta_new + P - A;
    size_t maxw = 0;
    for (size_t i = 0; i < nl; ++i) maxw = ls[i] > maxw ? ls[i] : maxw;
    double *buf = (double *)calloc(nl * maxw, sizeof(double));
    double *y[OR_MAX_LAYERS];
    for (size_t i = 0; i < nl; ++i) y[i] = buf + i * maxw;
    double surr = 0;
    for (size_t s = 0; s < n; ++s) {
        or_forward1(nl, ls, ac, W, B, obs + s * ls[0], y);
        double lld = 0;
        for (size_t i = 0; i < A; ++i) {
            double tx = (action[s * A + i] - mean[s * A + i]) / stdv[i];
            double tn = (action[s * A + i] - y[nl - 1][i]) / exp(logstd[i]);
            lld += tx * tx - tn * tn + log(stdv[i]) - logstd[i];
        }
        lld = lld * 0.5;
        surr += exp(lld) * adv[s];
    }
    free(buf);
    return surr;
}

/* One TRPO update (src/TRPO_Update.c:10-1011) with explicit settings (the reference
 * hard-wires maxiter 10, resth 1e-10, max_kl 0.01, max_bt 10, accept 0.1).  Outputs:
 * theta_out [P]; b_out / x_out [P] (policy gradient, CG step; may be NULL); scal[6] =
 * {shs, lagrange, gnorm, fval_before, expected_improve_rate, accepted k or -1};
 * are[3*max_bt] = actual/expected/ratio per evaluated backtrack; *evaluated. */
double oracle_update(size_t nl, const size_t *ls, const char *ac, const double *theta, const double *obs,
                     const double *mean, const double *action, const double *adv, const double *stdv, size_t n,
                     double damping, size_t maxiter, double resth, double max_kl, int max_bt, double accept,
                     double *theta_out, double *b_out, double *x_out, double *scal, double *are, int *evaluated,
                     int verbose) {
    const size_t P = oracle_num_params(ls, nl);
    double *b = (double *)calloc(P, sizeof(double)), *x = (double *)calloc(P, sizeof(double));
    double *z = (double *)calloc(P, sizeof(double)), *fullstep = (double *)calloc(P, sizeof(double));
    double *xnew = (double *)calloc(P, sizeof(double));
    double t0 = or_now(), adv_sum = 0;
    oracle_policy_grad(nl, ls, ac, theta, obs, mean, action, adv, n, 1, b, &adv_sum);
    if (oracle_cg(nl, ls, ac, theta, obs, n, stdv, damping, b, maxiter, resth, x, NULL, NULL, NULL, 1, verbose) < 0)
        return -1;
    oracle_fvp(nl, ls, ac, theta, obs, n, stdv, damping, x, z, 1);   /* :633-832 */
    double shs = 0;
    for (size_t i = 0; i < P; ++i) shs += z[i] * x[i];
    shs = shs * 0.5;
    if (verbose) printf("shs: %.14f\n", shs);
    double lm = sqrt(shs / max_kl);
    double gnorm = 0;
    for (size_t i = 0; i < P; ++i) gnorm += b[i] * b[i];
    gnorm = sqrt(gnorm);
    if (verbose) printf("lagrange multiplier: %.14f, gnorm: %.14f\n", lm, gnorm);
    for (size_t i = 0; i < P; ++i) fullstep[i] = x[i] / lm;
    double neggdotstepdir = 0;
    for (size_t i = 0; i < P; ++i) neggdotstepdir += b[i] * x[i];
    for (size_t i = 0; i < P; ++i) theta_out[i] = x[i];
    double rate = neggdotstepdir / lm;
    double fval = -adv_sum / (double)n;
    if (verbose) printf("fval before %.14e\n", fval);
    int acc = -1, ev = 0;
    for (int k = 0; k < max_bt; ++k) {
        double stepfrac = pow(0.5, (double)k);
        for (size_t i = 0; i < P; ++i) xnew[i] = theta[i] + stepfrac * fullstep[i];
        double surr = oracle_surrogate_sum(nl, ls, ac, xnew, obs, mean, action, adv, stdv, n);
        double newfval = -surr / (double)n;
        double actual = fval - newfval, expected = rate * stepfrac, ratio = actual / expected;
        if (verbose) printf("a/e/r %.14f / %.14f / %.14f\n", actual, expected, ratio);
        if (are) {
            are[3 * k] = actual;
            are[3 * k + 1] = expected;
            are[3 * k + 2] = ratio;
        }
        ev = k + 1;
        if (ratio > accept && actual > 0) {
            for (size_t i = 0; i < P; ++i) theta_out[i] = xnew[i];
            acc = k;
            break;
        }
    }
    double t1 = or_now();
    if (b_out) memcpy(b_out, b, P * sizeof(double));
    if (x_out) memcpy(x_out, x, P * sizeof(double));
    if (scal) {
        scal[0] = shs;
        scal[1] = lm;
        scal[2] = gnorm;
        scal[3] = fval;
        scal[4] = rate;
        scal[5] = acc;
    }
    if (evaluated) *evaluated = ev;
    free(b); free(x); free(z); free(fullstep); free(xnew);
    return t1 - t0;
}

/* Data file with every column (src/TRPO_Update.c:228-249); any output may be NULL. */
int oracle_load_rollout(const char *path, size_t nl, const size_t *ls, size_t n, double *obs, double *stdv,
                        double *mean, double *action, double *adv) {
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    const size_t O = ls[0], A = ls[nl - 1];
    double tmp;
    for (size_t s = 0; s < n; ++s) {
        for (size_t j = 0; j < A; ++j) {
            if (fscanf(f, "%lf", &tmp) != 1) goto bad;
            if (mean) mean[s * A + j] = tmp;
        }
        for (size_t j = 0; j < A; ++j) {
            if (fscanf(f, "%lf", &tmp) != 1) goto bad;
            if (stdv) stdv[j] = tmp;
        }
        for (size_t j = 0; j < O; ++j) {
            if (fscanf(f, "%lf", &tmp) != 1) goto bad;
            if (obs) obs[s * O + j] = tmp;
        }
        for (size_t j = 0; j < A; ++j) {
            if (fscanf(f, "%lf", &tmp) != 1) goto bad;
            if (action) action[s * A + j] = tmp;
        }
        if (fscanf(f, "%lf", &tmp) != 1) goto bad;
        if (adv) adv[s] = tmp;
    }
    fclose(f);
    return 0;
bad:
    fclose(f);
    return -1;
}

/* ------------------------------------------------------------------------- */
/* Value-baseline objective (src/TRPO_Baseline.c:29-240)                     */
/* ------------------------------------------------------------------------- */
/* x: NumParams (+ padding) parameters of the baseline MLP ls[0] = O + 1 (time feature), ...,
 * ls[nl-1] = 1.  observ [num_ep * ep_len][O], target [N].  g[n], predict[N] outputs.
 * Returns the objective 0.01 mean (pred - target)^2 + 0.001 |x|^2, or -1. */
double oracle_baseline_evaluate(size_t nl, const size_t *ls, const char *ac, const double *x, int n,
                                const double *observ, const double *target, size_t num_ep, size_t ep_len,
                                double *g, double *predict) {
    if (nl < 2 || nl > OR_MAX_LAYERS || ls[nl - 1] != 1) return -1;
    for (size_t i = 1; i < nl; ++i)
        if (ac[i] != 'l' && ac[i] != 't') return -1;
    const size_t O = ls[0] - 1, N = num_ep * ep_len;
    const size_t np = oracle_num_params(ls, nl) - 1;
    const double *W[OR_MAX_LAYERS], *B[OR_MAX_LAYERS];
    size_t Pfull;
    or_layers(nl, ls, x, W, B, &Pfull);
    size_t maxw = 0;
    for (size_t i = 0; i < nl; ++i) maxw = ls[i] > maxw ? ls[i] : maxw;
    double *buf = (double *)calloc(2 * nl * maxw, sizeof(double));
    double *y[OR_MAX_LAYERS], *gl[OR_MAX_LAYERS];
    for (size_t i = 0; i < nl; ++i) {
        y[i] = buf + (2 * i) * maxw;
        gl[i] = buf + (2 * i + 1) * maxw;
    }
    for (int i = 0; i < n; ++i) g[i] = 0;
    for (size_t ep = 0; ep < num_ep; ++ep) {
        for (size_t st = 0; st < ep_len; ++st) {
            const size_t pos = ep * ep_len + st;
            for (size_t i = 0; i < O; ++i) y[0][i] = observ[pos * O + i];
            y[0][O] = (double)st / (double)ep_len;                        /* :96-100 */
            for (size_t i = 0; i + 1 < nl; ++i) {                           /* :104-131 */
                for (size_t j = 0; j < ls[i + 1]; ++j) {
                    double v = B[i][j];
                    for (size_t k = 0; k < ls[i]; ++k) v += y[i][k] * W[i][k * ls[i + 1] + j];
                    if (ac[i + 1] == 't') v = tanh(v);
                    y[i + 1][j] = v;
                }
            }
            predict[pos] = y[nl - 1][0];                                    /* :135 */
            gl[nl - 1][0] = 0.02 * (predict[pos] - target[pos]);            /* :140 */
            size_t off = np;
            for (size_t i = nl - 1; i > 0; --i) {                           /* :143-205 */
                for (size_t j = 0; j < ls[i]; ++j)
                    if (ac[i] == 't') gl[i][j] = gl[i][j] * (1 - y[i][j] * y[i][j]);
                off -= ls[i - 1] * ls[i] + ls[i];
                for (size_t j = 0; j < ls[i - 1]; ++j)
                    for (size_t k = 0; k < ls[i]; ++k) g[off + j * ls[i] + k] += gl[i][k] * y[i - 1][j];
                for (size_t k = 0; k < ls[i]; ++k) g[off + ls[i - 1] * ls[i] + k] += gl[i][k];
                for (size_t j = 0; j < ls[i - 1]; ++j) {
                    double t = 0;
                    for (size_t k = 0; k < ls[i]; ++k) t += gl[i][k] * W[i - 1][j * ls[i] + k];
                    gl[i - 1][j] = t;
                }
            }
        }
    }
    for (size_t q = 0; q < np; ++q) g[q] = g[q] / (double)N + 0.002 * x[q];   /* :210-224 */
    double mse = 0;
    for (size_t i = 0; i < N; ++i) mse += 0.01 * (predict[i] - target[i]) * (predict[i] - target[i]);
    mse = mse / (double)N;
    double l2 = 0;
    for (size_t q = 0; q < np; ++q) l2 += x[q] * x[q];
    free(buf);
    return mse + 0.001 * l2;
}
