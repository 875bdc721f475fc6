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

int main(int argc, char **argv) {
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
        double t = FVPFast(prm, out, in, th);
        if (t < 0) return 1;
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
        if (is_time) {
            fprintf(stderr, "{\"compute_s\": %.9f, \"wall_s\": %.9f, \"threads\": %zu}\n", t, w1 - w0, th);
            return 0;
        }
        return write_vec(argv[11], out, P) ? 1 : 0;
    }
    fprintf(stderr, "unknown mode %s\n", mode);
    return 2;
}
