"""MI355X: size-independent properties of the Fisher-vector product and the CG solve at the
BASELINE sizes (armDOF_0 and 2x64, N = 50 000), where the fp64 oracle is too slow to run per case.

F + lambda I is symmetric positive definite, so for the device FVP z(v) = (F + lambda I) v:
  * linearity:  z(a u + b w) = a z(u) + b z(w)            (fp32 per-sample math: relative 1e-5)
  * symmetry:   u . z(w) = w . z(u)                       (relative 1e-5)
  * positivity: v . z(v) >= lambda |v|^2 > 0
  * the log-std block is exactly (2 + lambda) v            (src/TRPO_FVP.c:919-931, bit for bit)
and the CG step x for b satisfies |(F + lambda I) x - b| / |b| = sqrt(rdotr_final) / |b| as the
reference's recurrence reports it (src/TRPO_CG.c:56), within the fp32 FVP noise.
"""
import numpy as np
import pytest

import trpo_amd
from trpo_amd import synth

pytestmark = pytest.mark.gpu

SHAPES = {"armDOF_0": [15, 16, 16, 3], "2x64": [15, 64, 64, 3]}
N = 50_000
LAM = 0.1


def _ctx(layers, precision=None):
    th, obs = synth.make_theta(layers), synth.make_obs(N, layers[0])
    return trpo_amd.Context(layers, "lttl", th, obs, np.array([0.8, 1.0, 1.3]), LAM, precision=precision)


def _rel(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


@pytest.mark.parametrize("shape", list(SHAPES))
def test_fvp_linear_symmetric_positive(shape):
    layers = SHAPES[shape]
    P = synth.num_params(layers)
    rng = np.random.default_rng(11)
    u, w = rng.standard_normal(P), rng.standard_normal(P)
    a, b = 0.7, -1.9
    with _ctx(layers) as ctx:
        zu, zw, zc = ctx.fvp(u), ctx.fvp(w), ctx.fvp(a * u + b * w)
    assert _rel(zc, a * zu + b * zw) <= 1e-5
    assert abs(u @ zw - w @ zu) <= 1e-5 * abs(u @ zw)
    for v, z in ((u, zu), (w, zw)):
        assert v @ z >= LAM * (v @ v)
    A = layers[-1]
    np.testing.assert_array_equal(zu[-A:], 2.0 * u[-A:] + LAM * u[-A:])


@pytest.mark.parametrize("shape", list(SHAPES))
@pytest.mark.parametrize("precision", [None, "fp64"])
def test_cg_residual_matches_reported(shape, precision):
    layers = SHAPES[shape]
    P = synth.num_params(layers)
    b = synth.make_b(P)
    with _ctx(layers, precision) as ctx:
        x = ctx.cg(b, 10, 0.0)
        rr, _, iters = ctx.cg_history()
        res = ctx.fvp(x) - b
    assert iters == 10
    true_rel = np.linalg.norm(res) / np.linalg.norm(b)
    reported = np.sqrt(rr[iters]) / np.linalg.norm(b)
    # the recurrence residual tracks the true residual until it reaches the FVP's noise level
    tol = 1e-5 if precision is None else 1e-10
    assert abs(true_rel - reported) <= max(0.05 * reported, tol), (true_rel, reported)
    assert true_rel < 0.5                                         # the solve made progress
