"""The value-baseline fit driven by the caller's OWN optimiser: liblbfgs 1.10 as the reference vendors
it (src/lbfgs.c), called the way its trainer calls it (src/TRPO_Lightweight.c:347-349, :676:
default parameters, max_iterations = 25, no progress callback, lbfgs(PaddedParams, x, &fx, evaluate,
NULL, &BaselineParam, &param)).  oracle/_ref/libref_lbfgs.so holds that optimiser plus the
reference's own evaluate (src/TRPO_Baseline.c:29), built from the sources by `make -C oracle ref`
(oracle/lbfgs_fit.c is the thin caller).  The same optimiser binary then drives:
  * CPU: the reference's evaluate, and the clean-room oracle's evaluate through a ctypes callback;
  * GPU: libtrpo_mi355x.so's exported device evaluate -- the drop-in the unchanged trainer links.
The fit is a 25-step trajectory, so objective rounding (device: fp64, other summation order; DESIGN
§5.6) is amplified along it: the bound on the final parameters is relL2 <= 1e-8, on the objective
1e-10 relative, and the return code (stop reason) must agree.
"""
import ctypes as C
import os

import numpy as np
import pytest

import cases
import trpo_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_LBFGS = os.path.join(ROOT, "oracle", "_ref", "libref_lbfgs.so")
EVAL_T = C.CFUNCTYPE(C.c_double, C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_int, C.c_double)
LAYERS, ACF, NEP, EPLEN = [16, 16, 16, 1], "lttl", 20, 150     # the Lightweight trainer's baseline shape

needs_ref = pytest.mark.skipif(not os.path.exists(REF_LBFGS), reason="oracle/_ref not built (make -C oracle ref)")


def _ref():
    lib = C.CDLL(REF_LBFGS)
    lib.ref_lbfgs_fit.restype = C.c_int
    lib.ref_lbfgs_fit.argtypes = [C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_void_p, C.c_void_p,
                                  C.c_int]
    return lib


def _fit(ref, proc, param, x0):
    """One lbfgs() run from x0 (PaddedParams long) with the objective at address `proc`."""
    x = np.array(x0, np.float64)
    fx = C.c_double(0.0)
    rc = ref.ref_lbfgs_fit(x.size, x.ctypes.data_as(C.POINTER(C.c_double)), C.byref(fx), proc, C.byref(param), 25)
    return rc, fx.value, x


def _problem():
    """The trainer's TRPOBaselineParam (src/TRPO_MuJoCo.c:256-277) including the forward / backward
    scratch the reference's evaluate writes (LayerBase, GWBase, GBBase, GLayerBase); the device
    evaluate ignores the scratch."""
    x0, obs, tgt = trpo_amd.synth.make_baseline_problem(LAYERS, NEP, EPLEN)
    p = trpo_amd.make_baseline_param(LAYERS, ACF, obs, tgt, NEP, EPLEN)
    dpp = C.POINTER(C.c_double)
    lay = [np.zeros(s) for s in LAYERS]
    glay = [np.zeros(s) for s in LAYERS]
    gw = [np.zeros(w.size) for w in p.W]
    gb = [np.zeros(b.size) for b in p.B]
    arrs = [(dpp * len(a))(*[v.ctypes.data_as(dpp) for v in a]) for a in (lay, gw, gb, glay)]
    p.LayerBase, p.GWBase, p.GBBase, p.GLayerBase = [C.cast(a, C.POINTER(dpp)) for a in arrs]
    p._scratch = (lay, glay, gw, gb, arrs)
    return x0, obs, tgt, p


def _check(got, want):
    rc, fx, x = got
    rc_r, fx_r, x_r = want
    assert rc == rc_r
    assert abs(fx - fx_r) <= 1e-10 * abs(fx_r)
    assert cases.rel_l2(x, x_r) <= 1e-8


@needs_ref
def test_reference_lbfgs_drives_oracle_evaluate():
    """CPU: the harness itself -- liblbfgs on the reference's evaluate fits (rc >= 0, f falls), and the
    same optimiser on the clean-room oracle's evaluate follows the same trajectory."""
    import oracle
    ref = _ref()
    x0, obs, tgt, param = _problem()
    want = _fit(ref, C.cast(ref.evaluate, C.c_void_p), param, x0)
    f0 = oracle.baseline_evaluate(LAYERS, ACF, x0, obs, tgt, NEP, EPLEN)[0]
    assert want[0] >= 0 and want[1] < 0.9 * f0

    def cb(_inst, xp, gp, n, _step):
        f, g, _ = oracle.baseline_evaluate(LAYERS, ACF, np.ctypeslib.as_array(xp, (n,)).copy(), obs, tgt, NEP, EPLEN)
        np.ctypeslib.as_array(gp, (n,))[:] = g
        return f

    cfn = EVAL_T(cb)
    _check(_fit(ref, C.cast(cfn, C.c_void_p), param, x0), want)


@pytest.mark.gpu
@needs_ref
def test_reference_lbfgs_drives_device_evaluate():
    """GPU: the unchanged caller's optimiser on libtrpo_mi355x.so's exported evaluate (the symbol the
    trainer links instead of src/TRPO_Baseline.c's) ends where it ends on the reference's evaluate."""
    ref = _ref()
    x0, _, _, param = _problem()
    want = _fit(ref, C.cast(ref.evaluate, C.c_void_p), param, x0)
    _, _, _, param_dev = _problem()
    got = _fit(ref, C.cast(trpo_amd.lib().evaluate, C.c_void_p), param_dev, x0)
    _check(got, want)
    # the caller reads the fitted network back from W/B (src/TRPO_Lightweight.c:679-693): evaluate
    # left the last evaluated x there, as the reference's does
    assert np.all(np.isfinite(param_dev.W[0]))
    _time_fits(ref, param_dev, param, x0)


def _time_fits(ref, param_dev, param_ref, x0, reps=5):
    """C5's baseline fit timed with the caller's own optimiser (liblbfgs as the trainer
    calls it) on the device evaluate, beside the same optimiser on the reference's CPU evaluate (one
    host core).  bench.py may not run anything under oracle/ outside its CPU-baseline leg, so this GPU
    test is where the fit is timed; with TRPO_TIMING_OUT set, the medians go to that JSON file
    (profiles/r04_lbfgs_fit_timing.json)."""
    import json
    import time
    t_dev, t_ref = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        rc, _, _ = _fit(ref, C.cast(trpo_amd.lib().evaluate, C.c_void_p), param_dev, x0)
        t_dev.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        _fit(ref, C.cast(ref.evaluate, C.c_void_p), param_ref, x0)
        t_ref.append(time.perf_counter() - t0)
    out = {"what": "liblbfgs 1.10 lbfgs() (src/lbfgs.c, default parameters, max_iterations 25, the trainer's "
                   "call, src/TRPO_Lightweight.c:676) fitting the [16,16,16,1] baseline on 20 x 150 samples",
           "device_evaluate_fit_ms": 1e3 * float(np.median(t_dev)),
           "reference_cpu_evaluate_fit_ms_1core": 1e3 * float(np.median(t_ref)), "lbfgs_rc": int(rc), "reps": reps}
    print("[timing]", json.dumps(out))
    path = os.environ.get("TRPO_TIMING_OUT")
    if path:
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
