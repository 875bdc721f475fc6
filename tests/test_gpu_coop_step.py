"""MI355X: the cooperative path's distributed CG step (cg_dots_kernel + cg_axpy_kernel, 2x64-class nets)
when a solve stops early (src/TRPO_CG.c:65-103: `if (rdotr < ResidualTh) break`).

cg_axpy_kernel takes its stop test from the step's input state (rdotr < ResidualTh or iter >= MaxIter),
not from ctl->done, which block 0 of the same launch rewrites; a stopped step carries the state to
the next launch.  Checked: the iteration count and x against the oracle for solves that stop after a
few iterations, the launches after the stop leaving x untouched (an update-path CG with 1e-10 runs them
too), and bitwise repeatability of consecutive solves in one context.
"""
import numpy as np
import pytest

import cases
import oracle
import trpo_amd
from trpo_amd import synth

pytestmark = pytest.mark.gpu


def _problem(L, n, seed):
    th, obs = synth.make_theta(L, seed=seed), synth.make_obs(n, L[0], seed=seed + 1)
    return th, obs, np.linspace(0.8, 1.2, L[-1]), synth.make_b(synth.num_params(L), seed=seed + 2)


@pytest.mark.parametrize("scale,resth", [(1e-3, 1e-9), (1e-3, 1.2e-8), (1.0, 1e-4)])
def test_early_stop_matches_oracle(scale, resth):
    L = [15, 64, 64, 3]
    th, obs, std, b = _problem(L, 4096, 21)
    b = b * scale
    ref = oracle.cg(L, "lttl", th, obs, std, b, 10, resth)
    with trpo_amd.Context(L, "lttl", th, obs, std, 0.1) as ctx:
        assert ctx.kernel_name.endswith("coop"), ctx.kernel_name
        x = ctx.cg(b, 10, resth)
        rr, _, iters = ctx.cg_history()
    assert iters == ref["iters"]
    assert iters < 10
    assert cases.rel_l2(x, ref["x"]) <= 1e-4
    np.testing.assert_allclose(rr[:iters + 1], ref["rdotr"][:iters + 1], rtol=1e-2)


def test_repeated_solves_bitwise():
    L = [15, 64, 64, 3]
    th, obs, std, b = _problem(L, 50000, 9)
    with trpo_amd.Context(L, "lttl", th, obs, std, 0.1) as ctx:
        xs = [ctx.cg(b, 10, 0.0) for _ in range(3)] + [ctx.cg(b * 1e-3, 10, 1e-9), ctx.cg(b, 10, 0.0)]
    for x in (xs[1], xs[2], xs[4]):
        np.testing.assert_array_equal(x, xs[0])


def test_small_net_solves_after_early_stop_bitwise():
    """armDOF_0 (one-wave-per-tile kernels, fp64 atomic targets): the next solve's first atomic target is
    zeroed by the last step even when the solve has stopped early -- solves after early stops and after
    short solves give the bits of a fresh context's solve."""
    L = [15, 16, 16, 3]
    th, obs, std, b = _problem(L, 50000, 13)
    with trpo_amd.Context(L, "lttl", th, obs, std, 0.1) as ref:
        x_ref = ref.cg(b, 10, 0.0)
        x2_ref = ref.cg(b, 2, 0.0)
    with trpo_amd.Context(L, "lttl", th, obs, std, 0.1) as ctx:
        x_stop = ctx.cg(b, 10, 1e30)            # stops at iteration 0
        x_early = ctx.cg(b * 1e-3, 10, 1e-9)     # stops after a few iterations
        x_full = ctx.cg(b, 10, 0.0)
        x_two = ctx.cg(b, 2, 0.0)
        x_one = ctx.cg(b, 1, 0.0)
        x_again = ctx.cg(b, 10, 0.0)
    assert np.all(x_stop == 0.0)
    assert np.all(np.isfinite(x_early))
    np.testing.assert_array_equal(x_full, x_ref)
    np.testing.assert_array_equal(x_two, x2_ref)
    assert np.all(np.isfinite(x_one))
    np.testing.assert_array_equal(x_again, x_ref)
