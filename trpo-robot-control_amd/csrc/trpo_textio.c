/*
 * trpo_textio.c -- parsers of the reference's model and data text files (the host side of the
 * file-based entry points FVP / FVPFast / CG / TRPO_Update).  Plain C with no device dependency, so
 * `make -C oracle asan` builds it alone under -fsanitize=address,undefined and tests/test_textio.py
 * feeds it short, truncated, empty and garbage files (sanitizers on the CPU side).
 *
 * Semantics follow the reference's fscanf("%lf") loops: a file with fewer values than asked for
 * leaves the rest zero (its buffers are calloc'd, src/TRPO_FVP.c:591-664), and a token that is not a
 * number stops the parse for the rest of the file (fscanf never moves past it).
 */
#include "trpo_textio.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#define EXPORT __attribute__((visibility("default")))

EXPORT char *trpo_text_slurp(const char *path, size_t *len) {
    if (len) *len = 0;
    if (!path) return NULL;
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    /* regular files only: fopen succeeds on a directory, whose ftell then reports LONG_MAX (found by
     * the ASan build: a 2^63-byte malloc request) */
    struct stat st;
    if (fstat(fileno(f), &st) != 0 || !S_ISREG(st.st_mode) || st.st_size < 0) {
        fclose(f);
        return NULL;
    }
    const size_t sz = (size_t)st.st_size;
    char *buf = (char *)malloc(sz + 1);
    if (!buf) {
        fclose(f);
        return NULL;
    }
    const size_t got = fread(buf, 1, sz, f);      /* may be short if the file shrank meanwhile */
    fclose(f);
    buf[got] = 0;
    if (len) *len = got;
    return buf;
}

static int is_space(char c) { return c == ' ' || c == '\n' || c == '\t' || c == '\r' || c == '\v' || c == '\f'; }

/* one number at *pp (after whitespace); advances *pp and returns 1, or 0 at the end / a non-number */
static int next_double(const char **pp, double *v) {
    const char *p = *pp;
    while (is_space(*p)) ++p;
    *pp = p;
    if (!*p) return 0;
    char *e;
    *v = strtod(p, &e);
    if (e == p) return 0;
    *pp = e;
    return 1;
}

EXPORT size_t trpo_text_parse_doubles(const char *txt, double *out, size_t want) {
    size_t k = 0;
    const char *p = txt;
    while (k < want && next_double(&p, &out[k])) ++k;
    return k;
}

EXPORT int trpo_text_load_model(const char *path, size_t P, double *theta) {
    char *t = trpo_text_slurp(path, NULL);
    if (!t) {
        fprintf(stderr, "[ERROR] Cannot open Model File [%s]. \n", path ? path : "(null)");
        return -1;
    }
    const size_t got = trpo_text_parse_doubles(t, theta, P);
    free(t);
    for (size_t i = got; i < P; ++i) theta[i] = 0.0;      /* fscanf leaves calloc'd zeros */
    return 0;
}

EXPORT int trpo_text_load_data(const char *path, size_t O, size_t A, size_t n, double *obs, double *stdv,
                               double *mean, double *action, double *adv) {
    char *t = trpo_text_slurp(path, NULL);
    if (!t) {
        fprintf(stderr, "[ERROR] Cannot open Data File [%s]. \n", path ? path : "(null)");
        return -1;
    }
    const size_t row = 3 * A + O + 1;
    double *tmp = (double *)malloc(sizeof(double) * row);
    if (!tmp) {
        free(t);
        return -1;
    }
    const char *p = t;
    for (size_t s = 0; s < n; ++s) {
        size_t got = 0;
        while (got < row && next_double(&p, &tmp[got])) ++got;
        /* short row: the reference keeps what fscanf filled -- zeros, and the previous row's Std */
        for (size_t j = got; j < row; ++j) tmp[j] = (j >= A && j < 2 * A) ? stdv[j - A] : 0.0;
        if (mean) memcpy(mean + s * A, tmp, A * sizeof(double));
        memcpy(stdv, tmp + A, A * sizeof(double));
        memcpy(obs + s * O, tmp + 2 * A, O * sizeof(double));
        if (action) memcpy(action + s * A, tmp + 2 * A + O, A * sizeof(double));
        if (adv) adv[s] = tmp[3 * A + O];
    }
    free(tmp);
    free(t);
    return 0;
}
