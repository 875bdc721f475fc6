/* oracle/lbfgs_fit.c -- TEST INFRASTRUCTURE ONLY (built into oracle/_ref/libref_lbfgs.so).
 *
 * The caller side of the value-baseline fit as the reference's trainer runs it
 * (src/TRPO_Lightweight.c:347-349 and :676): liblbfgs 1.10's lbfgs() -- the copy vendored at
 * src/lbfgs.c, compiled unchanged beside this file -- with default parameters except
 * max_iterations = 25, no progress callback, and `evaluate` as the objective.  The objective is
 * passed in as a function pointer so one optimiser binary drives either the reference's own
 * evaluate (src/TRPO_Baseline.c:29, linked into the same library) or libtrpo_mi355x.so's device
 * evaluate; tests/test_gpu_baseline.py compares the two fits.  Nothing in the product links this.
 */
#include <stddef.h>
#include "lbfgs.h"

int ref_lbfgs_fit(int n, double *x, double *fx, lbfgs_evaluate_t proc, void *instance, int max_iterations)
{
    lbfgs_parameter_t param;
    lbfgs_parameter_init(&param);
    param.max_iterations = max_iterations;
    return lbfgs(n, x, fx, proc, NULL, instance, &param);
}
