"""The fp32 stall guard: a CG solve in which a Ritz value converges to machine
precision -- where the reference's own fp64 CG (src/TRPO_CG.c:65-103) loses orthogonality, so its step is
its rounding's and not the exact-arithmetic step the reorthogonalised fp32 solve converges to -- is
repeated in fp64 on a twin of the context, and trpo_ctx_cg_status reports it.  Checked: which solves
trigger it (the iterate-past-convergence fixture and random draw 23 do, the N = 50k headline does not),
that the re-solve is the fp64 mode's result bit for bit, and that the guard switched off leaves the fp32
step (draw 23: 1.2e-3 from the reference, the reason the guard exists)."""
import os

import numpy as np
import pytest

import cases
import oracle
import trpo_amd
from trpo_amd import synth

pytestmark = pytest.mark.gpu


def _ctx(x, **kw):
    return trpo_amd.Context(x["layers"], x["acfunc"], x["theta"], x["obs"], x["std"], x["damping"], **kw)


def test_headline_solve_is_not_resolved():
    c = cases.case("syn_arm_cg_n50000")
    x = cases.inputs(c)
    with _ctx(x) as ctx:
        got = ctx.cg(x["vin"], c["maxiter"], c["resth"])
        st = ctx.cg_status()
    assert not st["fp64_rerun"] and st["ritz_residual"] > 1e-13, st
    assert cases.rel_l2(got, cases.expected(c)) <= 1e-6


def test_past_convergence_solve_is_resolved_in_fp64(monkeypatch):
    """fix_cg_n3150_th0 iterates past convergence (rdotr 1e-14): its Ritz values are converged to 1e-17."""
    c = cases.case("fix_cg_n3150_th0")
    x = cases.inputs(c)
    with _ctx(x) as ctx:
        got = ctx.cg(x["vin"], c["maxiter"], c["resth"])
        st = ctx.cg_status()
        rr, _, it = ctx.cg_history()
        np.testing.assert_array_equal(ctx.download_x(), got)   # the device slot holds the returned x
    assert st["fp64_rerun"] and st["ritz_residual"] < 1e-15, st
    with _ctx(x, precision="fp64") as c64:
        want = c64.cg(x["vin"], c["maxiter"], c["resth"])
        rr64, _, it64 = c64.cg_history()
    np.testing.assert_array_equal(got, want)            # the twin IS the fp64 mode
    np.testing.assert_array_equal(rr, rr64)             # and the history the caller sees is the fp64 one
    assert it == it64 == c["iters"]
    assert cases.rel_l2(got, cases.expected(c)) <= 1e-5
    monkeypatch.setenv("TRPO_RITZ_RERUN", "0")
    with _ctx(x) as ctx:
        g32 = ctx.cg(x["vin"], c["maxiter"], c["resth"])
        assert not ctx.cg_status()["fp64_rerun"]
    assert cases.rel_l2(g32, cases.expected(c)) <= 1e-4  # the fp32 solve alone is within the bound too


def test_stalled_update_draw23(monkeypatch):
    from test_gpu_random_shapes import _draw
    layers, acts, n, std = _draw(23)
    th = synth.make_theta(layers, seed=123)
    obs = synth.make_obs(n, layers[0], seed=223)
    mean, action, adv = synth.make_rollout(layers, acts, th, obs, std, seed=523)
    ref = oracle.update(layers, acts, th, obs, mean, action, adv, std, 0.1)
    with trpo_amd.Context(layers, acts, th, obs, std, 0.1) as ctx:
        ctx.set_rollout(mean, action, adv)
        r = ctx.update()
    assert r["fp64_rerun"] and r["ritz_residual"] < 1e-15, (r["ritz_residual"], r["fp64_rerun"])
    assert cases.rel_l2(r["x"], ref["x"]) <= 1e-4
    monkeypatch.setenv("TRPO_RITZ_RERUN", "0")
    with trpo_amd.Context(layers, acts, th, obs, std, 0.1) as ctx:
        ctx.set_rollout(mean, action, adv)
        r32 = ctx.update()
    assert not r32["fp64_rerun"]
    assert cases.rel_l2(r32["x"], ref["x"]) > 1e-4        # why the guard exists: 1.2e-3


def test_twin_follows_the_context(monkeypatch):
    """set_theta / set_damping after a re-solve: the next re-solve uses the new problem (the twin is
    rebuilt or updated), never a stale copy."""
    c = cases.case("fix_cg_n3150_th0")
    x = cases.inputs(c)
    th2 = x["theta"] * 1.01
    with _ctx(x) as ctx:
        ctx.cg(x["vin"], c["maxiter"], c["resth"])
        assert ctx.cg_status()["fp64_rerun"]
        ctx.set_theta(th2)
        ctx.set_damping(0.2)
        got = ctx.cg(x["vin"], c["maxiter"], c["resth"])
        st = ctx.cg_status()
    x2 = dict(x, theta=th2, damping=0.2)
    with _ctx(x2, precision="fp64") as c64:
        want = c64.cg(x["vin"], c["maxiter"], c["resth"])
    if st["fp64_rerun"]:
        np.testing.assert_array_equal(got, want)
    else:
        assert cases.rel_l2(got, want) <= 1e-4
