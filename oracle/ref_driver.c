/*
 * ref_driver.c -- TEST INFRASTRUCTURE ONLY (our own main, not reference code).
 *
 * Drives the reference's UNCHANGED src/TRPO_FVP.c, src/TRPO_CG.c,
 * src/TRPO_Util.c and src/TRPO_Update.c, compiled straight from /root/reference by oracle/Makefile
 * into oracle/_ref/.  Used (a) by tests/golden/make_goldens.py to produce the
 * golden vectors committed under tests/golden/, and (b) by bench.py's
 * cpu_baseline leg ("kind": "reference") when oracle/_ref/ is present.
 *
 *   ref_driver fvp  MODEL DATA N LAYERS ACFUNC DAMPING VIN  OUT [THREADS]
 *   ref_driver cg   MODEL DATA N LAYERS ACFUNC DAMPING BIN  MAXITER RESTH OUT [THREADS]
 *   ref_driver time MODEL DATA N LAYERS ACFUNC DAMPING BIN  MAXITER RESTH [THREADS]
 *   ref_driver update MODEL DATA N LAYERS ACFUNC DAMPING OUT [THREADS]
 *   ref_driver baseline LAYERS ACFUNC NUMEP EPLEN OBSFILE TARGETFILE XFILE OUT
 *       (the reference's evaluate(), src/TRPO_Baseline.c:29; OUT = g [PaddedParams] then
 *        Predict [N]; the objective is printed as "f %.17g")
 *
 * LAYERS is a comma list (e.g. 15,16,16,3); ACFUNC a string (e.g. lttl).
 * Vectors are text, one %.17g value per line.  The reference's own stdout
 * (CG progress lines, per-sample mean checks) is left on stdout.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>

#include "TRPO.h"
#include "lbfgs.h"

lbfgsfloatval_t evaluate(void *param_in, const lbfgsfloatval_t *x, lbfgsfloatval_t *g, const int n,
                         const lbfgsfloatval_t step);   /* defined in src/TRPO_Baseline.c, no header prototype */

static size_t parse_layers(const char *s, size_t *ls) {
    size_t n = 0;
    char *dup = strdup(s), *tok = strtok(dup, ",");
    while (tok && n < 16) {
        ls[n++] = (size_t)strtoull(tok, NULL, 10);
        tok = strtok(NULL, ",");
    }
    free(dup);
    return n;
}

static int read_vec(const char *path, double *v, size_t n) {
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    for (size_t i = 0; i < n; ++i)
        if (fscanf(f, "%lf", &v[i]) != 1) {
            fclose(f);
            return -1;
        }
    fclose(f);
    return 0;
}

static int write_vec(const char *path, const double *v, size_t n) {
    FILE *f = fopen(path, "w");
    if (!f) return -1;
    for (size_t i = 0; i < n; ++i) fprintf(f, "%.17g\n", v[i]);
    fclose(f);
    return 0;
}

static double wall(void) {
    struct timeval tv;
    gettimeofday(&tv, NULL);
    return tv.tv_sec + 1e-6 * tv.tv_usec;
}

static int run_baseline(int argc, char **argv) {
    if (argc < 10) return 2;
    size_t ls[16];
    const size_t nl = parse_layers(argv[2], ls);
    char acf[17] = {0};
    strncpy(acf, argv[3], 16);
    const size_t nep = (size_t)strtoull(argv[4], NULL, 10), eplen = (size_t)strtoull(argv[5], NULL, 10);
    const size_t N = nep * eplen, O = ls[0] - 1;
    const size_t np = NumParamsCalc(ls, nl) - 1;
    const int padded = (int)((np + 15) / 16 * 16);
    double *obs = calloc(N * O, sizeof(double)), *tgt = calloc(N, sizeof(double));
    double *pred = calloc(N, sizeof(double)), *x = calloc(padded, sizeof(double)), *g = calloc(padded, sizeof(double));
    if (read_vec(argv[6], obs, N * O) || read_vec(argv[7], tgt, N) || read_vec(argv[8], x, np)) return 1;
    double *W[16], *B[16], *Lay[16], *GW[16], *GB[16], *GL[16];
    for (size_t i = 0; i + 1 < nl; ++i) {
        W[i] = calloc(ls[i] * ls[i + 1], sizeof(double));
        B[i] = calloc(ls[i + 1], sizeof(double));
        GW[i] = calloc(ls[i] * ls[i + 1], sizeof(double));
        GB[i] = calloc(ls[i + 1], sizeof(double));
    }
    for (size_t i = 0; i < nl; ++i) {
        Lay[i] = calloc(ls[i], sizeof(double));
        GL[i] = calloc(ls[i], sizeof(double));
    }
    TRPOBaselineParam bp;             /* filled like src/TRPO_MuJoCo.c:256-277 */
    memset(&bp, 0, sizeof bp);
    bp.NumLayers = nl;
    bp.ObservSpaceDim = O;
    bp.NumEpBatch = nep;
    bp.EpLen = eplen;
    bp.NumSamples = N;
    bp.NumParams = np;
    bp.PaddedParams = padded;
    bp.AcFunc = acf;
    bp.LayerSizeBase = ls;
    bp.WBase = W;
    bp.BBase = B;
    bp.LayerBase = Lay;
    bp.GWBase = GW;
    bp.GBBase = GB;
    bp.GLayerBase = GL;
    bp.Observ = obs;
    bp.Target = tgt;
    bp.Predict = pred;
    double f = evaluate(&bp, x, g, padded, 1.0);
    printf("f %.17g\n", f);
    FILE *out = fopen(argv[9], "w");
    if (!out) return 1;
    for (int i = 0; i < padded; ++i) fprintf(out, "%.17g\n", g[i]);
    for (size_t i = 0; i < N; ++i) fprintf(out, "%.17g\n", pred[i]);
    fclose(out);
    return 0;
}

int main(int argc, char **argv) {
    if (argc > 1 && !strcmp(argv[1], "baseline")) return run_baseline(argc, argv);
    if (argc < 9) {
        fprintf(stderr, "usage: see header of ref_driver.c\n");
        return 2;
    }
    const char *mode = argv[1];
    size_t ls[16];
    char acf[17] = {0};
    TRPOparam prm;
    memset(&prm, 0, sizeof prm);
    prm.ModelFile = argv[2];
    prm.DataFile = argv[3];
    prm.NumSamples = (size_t)strtoull(argv[4], NULL, 10);
    prm.NumLayers = parse_layers(argv[5], ls);
    strncpy(acf, argv[6], 16);
    prm.AcFunc = acf;
    prm.LayerSize = ls;
    prm.CG_Damping = atof(argv[7]);
    const size_t P = NumParamsCalc(ls, prm.NumLayers);
    double *in = calloc(P, sizeof(double)), *out = calloc(P, sizeof(double));
    if (!strcmp(mode, "update")) {       /* TRPO_Update prints shs / lagrange / a/e/r itself */
        size_t th = argc > 9 ? (size_t)atoi(argv[9]) : 1;
        double w0 = wall();
        double t = TRPO_Update(prm, out, th);
        double w1 = wall();
        if (t < 0) return 1;
        fprintf(stderr, "{\"compute_s\": %.9f, \"wall_s\": %.9f, \"threads\": %zu}\n", t, w1 - w0, th);
        return write_vec(argv[8], out, P) ? 1 : 0;
    }
    if (read_vec(argv[8], in, P)) {
        fprintf(stderr, "cannot read %s\n", argv[8]);
        return 1;
    }
    if (!strcmp(mode, "fvp")) {
        size_t th = argc > 10 ? (size_t)atoi(argv[10]) : 1;
        double w0 = wall();
        double t = FVPFast(prm, out, in, th);
        double w1 = wall();
        if (t < 0) return 1;
        fprintf(stderr, "{\"compute_s\": %.9f, \"wall_s\": %.9f, \"threads\": %zu}\n", t, w1 - w0, th);
        return write_vec(argv[9], out, P) ? 1 : 0;
    }
    if (!strcmp(mode, "cg") || !strcmp(mode, "time")) {
        size_t maxiter = (size_t)strtoull(argv[9], NULL, 10);
        double resth = atof(argv[10]);
        int is_time = !strcmp(mode, "time");
        size_t th = 1;
        if (!is_time && argc > 12) th = (size_t)atoi(argv[12]);
        if (is_time && argc > 11) th = (size_t)atoi(argv[11]);
        double w0 = wall();
        double t = CG(prm, out, in, maxiter, resth, th);
        double w1 = wall();
        if (t < 0) return 1;
        fprintf(stderr, "{\"compute_s\": %.9f, \"wall_s\": %.9f, \"threads\": %zu}\n", t, w1 - w0, th);
        if (is_time) return 0;
        return write_vec(argv[11], out, P) ? 1 : 0;
    }
    fprintf(stderr, "unknown mode %s\n", mode);
    return 2;
}
