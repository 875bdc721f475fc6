"""MI355X: the armDOF_0 FVP and CG at the C4 sweep's batch sizes (and the 2x64 cooperative FVP) (N = 500k and 4M), where
the throughput-regime kernel variants run (the narrow-output twin picked by tiles per wave, §5.1b)
and the fp64 oracle is far too slow.  Size-independent properties only:
  * linearity, symmetry, positivity and the exact log-std block, as tests/test_gpu_properties.py at 50k;
  * sample-shard decomposition: the FVP is a mean over samples (src/TRPO_FVP.c:771-931), so the
    un-normalised weight block over all N equals the sum of the blocks of two contexts holding the
    halves of the same seeded sample stream -- (z - lambda v) N = (z1 - lambda v) N1 + (z2 - lambda v) N2
    -- which checks the full-size cross-block accumulation against independent smaller launches
    (fp32 block partials added in fp64, different block partition: measured 3.5e-9 for armDOF_0 at 500k
    and 4M, 3.4e-9 / 6.8e-9 for the 2x64 cooperative slab path at 50k / 500k,
    tools/diag/large_n_decomposition.py; bound 1e-7);
  * the CG step's true residual against the recurrence's reported one (src/TRPO_CG.c:56).
"""
import numpy as np
import pytest

import trpo_amd
from trpo_amd import synth

pytestmark = pytest.mark.gpu

ARM = [15, 16, 16, 3]
LAM = 0.1
STD = np.array([0.8, 1.0, 1.3])
SIZES = [500_000, 4_000_000]


def _ctx(n, start=0, layers=ARM):
    return trpo_amd.Context(layers, "lttl", synth.make_theta(layers), synth.make_obs(n, layers[0], start=start), STD,
                            LAM)


def _rel(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


W64 = [15, 64, 64, 3]
CASES = [(ARM, n) for n in SIZES] + [(W64, 50_000), (W64, 500_000)]   # + the cooperative slab path (2x64)


@pytest.mark.parametrize("layers,n", CASES, ids=["%s-%d" % ("x".join(map(str, l)), n) for l, n in CASES])
def test_fvp_properties_and_shard_decomposition(layers, n):
    P = synth.num_params(layers)
    rng = np.random.default_rng(23)
    u, w = rng.standard_normal(P), rng.standard_normal(P)
    a, b = -0.6, 1.3
    with _ctx(n, layers=layers) as ctx:
        zu, zw, zc = ctx.fvp(u), ctx.fvp(w), ctx.fvp(a * u + b * w)
    assert _rel(zc, a * zu + b * zw) <= 1e-5
    assert abs(u @ zw - w @ zu) <= 1e-5 * abs(u @ zw)
    for v, z in ((u, zu), (w, zw)):
        assert v @ z >= LAM * (v @ v)
    A = layers[-1]
    np.testing.assert_array_equal(zu[-A:], 2.0 * u[-A:] + LAM * u[-A:])
    n1 = n // 2 + 37                                   # uneven halves, not tile multiples
    with _ctx(n1, layers=layers) as c1:
        z1 = c1.fvp(u)
    with _ctx(n - n1, start=n1, layers=layers) as c2:
        z2 = c2.fvp(u)
    nw = P - A
    full = (zu[:nw] - LAM * u[:nw]) * n
    parts = (z1[:nw] - LAM * u[:nw]) * n1 + (z2[:nw] - LAM * u[:nw]) * (n - n1)
    assert _rel(full, parts) <= 1e-7


def test_cg_residual_matches_reported_4m():
    P = synth.num_params(ARM)
    b = synth.make_b(P)
    with _ctx(SIZES[-1]) as ctx:
        x = ctx.cg(b, 10, 0.0)
        rr, _, iters = ctx.cg_history()
        res = ctx.fvp(x) - b
    assert iters == 10
    true_rel = np.linalg.norm(res) / np.linalg.norm(b)
    reported = np.sqrt(rr[iters]) / np.linalg.norm(b)
    assert abs(true_rel - reported) <= max(0.05 * reported, 1e-5), (true_rel, reported)
    assert true_rel < 0.5
