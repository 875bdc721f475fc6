"""TEST INFRASTRUCTURE, run by bench.py as a child process for config C5's baseline fit.

The value-baseline fit a trainer runs per iteration, driven by the caller's OWN optimiser: liblbfgs 1.10
as the reference vendors it (src/lbfgs.c, in oracle/_ref/libref_lbfgs.so), called as
src/TRPO_Lightweight.c:347-349, :676 call it (default parameters, max_iterations 25), on
libtrpo_mi355x.so's exported device `evaluate`; the same optimiser on the reference's CPU `evaluate`
(one host core) is timed beside it.  Reuses tests/test_lbfgs_caller.py's harness (which also checks the
two fits agree).  Prints one JSON line on stdout: the medians of `reps` fits.
    python tests/lbfgs_fit_child.py [reps]
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(ROOT, "trpo-robot-control_amd"), HERE]


def main():
    import contextlib
    import io
    import trpo_amd
    trpo_amd.lib()
    import test_lbfgs_caller as t
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    ref = t._ref()
    x0, _, _, param_ref = t._problem()
    _, _, _, param_dev = t._problem()
    want = t._fit(ref, t.C.cast(ref.evaluate, t.C.c_void_p), param_ref, x0)
    got = t._fit(ref, t.C.cast(trpo_amd.lib().evaluate, t.C.c_void_p), param_dev, x0)
    t._check(got, want)                         # same stop reason, objective and parameters
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        t._time_fits(ref, param_dev, param_ref, x0, reps=reps)
    line = [l for l in buf.getvalue().splitlines() if l.startswith("[timing] ")][-1]
    out = json.loads(line[len("[timing] "):])
    out["fit_matches_reference_fit"] = True
    print(json.dumps(out))


if __name__ == "__main__":
    main()
