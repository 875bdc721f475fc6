"""Line-search surrogate sums (src/TRPO_Update.c:951-981) through trpo_ctx_surrogate.

The wide 3-weight-layer policies (hidden widths 17..64, e.g. the 2x64 MLP) run on the fp64 MFMA kernel
(surr_mfma_kernel: one wave per 16-sample tile, activations in the accumulator registers); the
one-lane-per-sample fp64 kernel is the TRPO_SURR_GENERIC=1 path, and widths <= 16 take the register
kernel.  Every path is checked against the clean-room oracle's fp64 sum (pinned bit-exact to the
reference's TRPO_Update goldens) at 1e-12 relative: the MFMA forward rounds its dot products in a
different order (measured ~1e-15), not at lower precision.
"""
import numpy as np
import pytest

import oracle
import trpo_amd
from trpo_amd import synth

pytestmark = pytest.mark.gpu

TOL = 1e-12


def _problem(L, n, seed=5):
    th = synth.make_theta(L)
    obs = synth.make_obs(n, L[0])
    std = np.linspace(0.7, 1.3, L[-1])
    mean, action, adv = synth.make_rollout(L, "lttl", th, obs, std)
    rng = np.random.default_rng(seed)
    fs = 0.05 * rng.standard_normal(th.size) * np.abs(th).mean()
    return th, obs, std, mean, action, adv, fs


def _oracle_sums(L, th, obs, std, mean, action, adv, fs, k0, nk):
    return np.array([oracle.surrogate_sum(L, "lttl", th + 0.5 ** (k0 + j) * fs, obs, mean, action, adv, std)
                     for j in range(nk)])


@pytest.mark.parametrize("L", [[15, 64, 64, 3], [15, 32, 32, 3], [15, 48, 48, 3], [20, 64, 64, 5],
                               [15, 16, 16, 3]])
@pytest.mark.parametrize("n", [1, 17, 1000, 4099])
def test_surrogate_matches_oracle(L, n):
    th, obs, std, mean, action, adv, fs = _problem(L, n)
    with trpo_amd.Context(L, "lttl", th, obs, std, 0.1) as ctx:
        ctx.set_rollout(mean, action, adv)
        s = ctx.surrogate(fs, 0, 5)
        s2 = ctx.surrogate(fs, 3, 2)
    ref = _oracle_sums(L, th, obs, std, mean, action, adv, fs, 0, 5)
    np.testing.assert_allclose(s, ref, rtol=TOL, atol=TOL * np.abs(ref).max())
    np.testing.assert_allclose(s2, ref[3:5], rtol=TOL, atol=TOL * np.abs(ref).max())


def test_surrogate_mfma_matches_generic(monkeypatch):
    """2x64 at N = 50 000: the MFMA kernel against the one-lane-per-sample fp64 kernel."""
    L, n = [15, 64, 64, 3], 50000
    th, obs, std, mean, action, adv, fs = _problem(L, n)
    out = []
    for generic in ("0", "1"):
        monkeypatch.setenv("TRPO_SURR_GENERIC", generic)
        with trpo_amd.Context(L, "lttl", th, obs, std, 0.1) as ctx:
            ctx.set_rollout(mean, action, adv)
            out.append(ctx.surrogate(fs, 0, 10))
    np.testing.assert_allclose(out[0], out[1], rtol=TOL)
