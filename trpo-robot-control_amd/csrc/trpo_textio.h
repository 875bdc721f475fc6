/*
 * trpo_textio.h -- the reference's text formats (internal to libtrpo_mi355x.so; exported with the
 * trpo_text_ prefix so the CPU tests can drive them, also under AddressSanitizer + UBSan).
 */
#ifndef TRPO_TEXTIO_H
#define TRPO_TEXTIO_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* whole file, NUL-terminated (len may be NULL); NULL if it cannot be opened or read */
char *trpo_text_slurp(const char *path, size_t *len);
/* up to `want` doubles from whitespace-separated text, fscanf("%lf") semantics: stops at the end or
 * at the first token that is not a number; returns how many were parsed */
size_t trpo_text_parse_doubles(const char *txt, double *out, size_t want);
/* model file (src/TRPO_FVP.c:670-699): theta[P]; entries the file lacks are 0 */
int trpo_text_load_model(const char *path, size_t P, double *theta);
/* data file (src/TRPO_FVP.c:731-762, src/TRPO_Update.c:228-249): first n rows of
 * Mean[A] Std[A] Obs[O] Action[A] Adv; stdv = the Std of the last row; mean / action / adv may be NULL */
int trpo_text_load_data(const char *path, size_t O, size_t A, size_t n, double *obs, double *stdv, double *mean,
                        double *action, double *adv);

#ifdef __cplusplus
}
#endif
#endif
