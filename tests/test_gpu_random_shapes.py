"""Randomised shape sweep: FVP, CG and the TRPO update on the device against the clean-room oracle
(pinned to the reference's TRPO_FVP.c / TRPO_CG.c / TRPO_Update.c) for policies drawn at random
across every kernel family -- the one-wave-per-tile kernel (widths <= 16 per tile), the cooperative
kernel (equal hidden widths 32 / 48 / 64), the generic kernel (deeper nets, wider layers) -- with
random activations, sample counts that are not multiples of 16 and sigma != 1.

Tolerances as the golden tests: FVP relative L2 <= 1e-5, CG / update step <= 1e-4 (fp32 FVP,
reorthogonalised fp64 CG; tests/test_gpu_parity.py), policy gradient <= 2e-6.  Every draw also runs in
the fp64 precision mode (tile shapes on the cooperative fp64 kernel, the rest on the generic kernel's
fp64 instantiation): FVP <= 1e-12, update step <= 1e-4.
Draw 23 ([4,54,26,17,5] 'lslll', generic kernel) is the stalled solve: the reference's CG on that
update's right-hand side stalls at iterations 8 -> 9 (rdotr 3.97e-8 -> 3.92e-8) and then drops 160x in
its tenth step -- its own fp64 residuals have lost orthogonality, so the step it returns is not the
exact-arithmetic CG step, and the reorthogonalised fp32 solve lands 1.2e-3 from it
(profiles/r04_cg_history_fp32_vs_ref.log).  The fp32 stall guard (trpo_ctx_cg_status)
sees a Ritz value of that solve converged to below machine precision (7e-17; every other draw and golden
>= 1.6e-15, tools/diag/ritz_probe.py) -- where, by Paige's theory, plain CG's residuals lose
orthogonality -- and repeats that update in fp64 (the reference's arithmetic, 1.0e-5), so every draw's
fp32 update is asserted at 1e-4, and draw 23 must have been re-solved.
The draws are seeded, so a failure names a reproducible
configuration.
"""
import numpy as np
import pytest

import cases
import oracle
import trpo_amd
from trpo_amd import synth

pytestmark = pytest.mark.gpu

ACTS = "ltso"                     # linear, tanh, sigmoid, 0.1 x (the reference's four kinds)
STALLED = {23}                     # the fp32 stall guard must re-solve these in fp64 (module docstring)


def _draw(seed):
    rng = np.random.default_rng(seed)
    kind = seed % 3
    L0 = int(rng.integers(3, 33))
    A = int(rng.integers(1, 7))
    if kind == 0:                                  # small hidden layers: one-wave-per-tile kernel
        h1, h2 = int(rng.integers(4, 33)), int(rng.integers(4, 33))
        layers = [L0, h1, h2, A]
    elif kind == 1:                                # equal wide hidden layers: cooperative kernel
        h = int(rng.choice([32, 48, 64]))
        layers = [L0, h, h, A]
    else:                                          # deeper / wider: generic kernel
        depth = int(rng.integers(2, 5))
        layers = [L0] + [int(rng.integers(8, 80)) for _ in range(depth)] + [A]
    acts = "l" + "".join(rng.choice(list(ACTS), size=len(layers) - 2)) + str(rng.choice(["l", "l", "t"]))
    n = int(rng.integers(17, 3000))
    std = rng.uniform(0.5, 1.6, size=A)
    return layers, acts, n, std


@pytest.mark.parametrize("seed", range(36))
def test_random_policy_fvp_cg_update(seed):
    layers, acts, n, std = _draw(seed)
    th = synth.make_theta(layers, seed=100 + seed)
    obs = synth.make_obs(n, layers[0], seed=200 + seed)
    P = synth.num_params(layers)
    v, b = synth.make_v(P, seed=300 + seed), synth.make_b(P, seed=400 + seed)
    zr, _ = oracle.fvp(layers, acts, th, obs, std, v)
    xr = oracle.cg(layers, acts, th, obs, std, b, 10, 0.0)["x"]
    mean, action, adv = synth.make_rollout(layers, acts, th, obs, std, seed=500 + seed)
    ref = oracle.update(layers, acts, th, obs, mean, action, adv, std, 0.1)
    bref, _ = oracle.policy_grad(layers, acts, th, obs, mean, action, adv)
    with trpo_amd.Context(layers, acts, th, obs, std, 0.1) as ctx:
        kname = ctx.kernel_name
        z = ctx.fvp(v)
        x = ctx.cg(b, 10, 0.0)
        ctx.set_rollout(mean, action, adv)
        r = ctx.update()
    what = "%s %s n=%d kernel=%s" % (layers, acts, n, kname)
    assert cases.rel_l2(z, zr) <= 1e-5, what
    assert cases.rel_l2(x, xr) <= 1e-4, what
    assert cases.rel_l2(r["b"], bref) <= 2e-6, what
    assert r["accepted"] == ref["accepted"], what
    assert cases.rel_l2(r["x"], ref["x"]) <= 1e-4, (what, r["ritz_residual"], r["fp64_rerun"])
    if ref["accepted"] >= 0:
        assert cases.rel_l2(r["theta"] - th, ref["theta"] - th) <= 1e-4, what
    if seed in STALLED:
        assert r["fp64_rerun"], (what, r["ritz_residual"])
    with trpo_amd.Context(layers, acts, th, obs, std, 0.1, precision="fp64") as c64:
        z64 = c64.fvp(v)
        c64.set_rollout(mean, action, adv)
        r64 = c64.update()
    assert cases.rel_l2(z64, zr) <= 1e-12, what + " fp64"
    assert r64["accepted"] == ref["accepted"], what + " fp64"
    assert cases.rel_l2(r64["x"], ref["x"]) <= 1e-4, what + " fp64"
    if ref["accepted"] >= 0:
        assert cases.rel_l2(r64["theta"] - th, ref["theta"] - th) <= 1e-4, what + " fp64"
