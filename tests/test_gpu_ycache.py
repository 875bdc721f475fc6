"""MI355X: the forward-activation cache of the tile kernels (one-wave-per-tile and cooperative).

Within a CG solve theta and the observations are fixed, so the first FVP (MODE 0) writes the
per-tile forward activations y1, y2 (y3) and every later FVP (MODE 2) reads them and recomputes
only the R chains.  The cached path must give BIT-IDENTICAL results to the recomputing one
(TRPO_YCACHE=0), and must never serve activations of an older theta or observation set.
Parity against the reference goldens is covered by test_gpu_parity.py (same tolerances).
"""
import numpy as np
import pytest

import cases
import oracle
import trpo_amd
from trpo_amd import synth

pytestmark = pytest.mark.gpu

FVP_TOL = 1e-5


def _ctx(x, **kw):
    return trpo_amd.Context(x["layers"], x["acfunc"], x["theta"], x["obs"], x["std"], x["damping"], **kw)


def _both(monkeypatch, make):
    """(cached, recomputing) results of make(ctx) on two contexts."""
    monkeypatch.setenv("TRPO_YCACHE", "0")
    ref = make()
    monkeypatch.delenv("TRPO_YCACHE")
    return make(), ref


@pytest.mark.parametrize("name", ["fix_fvp_n3150", "fix_fvp_n17", "fix_fvp_n1", "syn_sigma_fvp", "syn_acts_fvp"])
def test_repeated_fvp_bitwise_equal_and_golden(name, monkeypatch):
    c = cases.case(name)
    x = cases.inputs(c)

    def run():
        with _ctx(x) as ctx:
            return [ctx.fvp(x["vin"]) for _ in range(3)]   # 1st writes the cache, 2nd/3rd read it

    got, ref = _both(monkeypatch, run)
    for a in got + ref:
        np.testing.assert_array_equal(a, ref[0])
    assert cases.rel_l2(got[2], cases.expected(c)) <= FVP_TOL


@pytest.mark.parametrize("name", ["fix_cg_n3150_th0", "syn_sigma_cg", "syn_arm_cg_n50000"])
def test_cg_bitwise_equal(name, monkeypatch):
    c = cases.case(name)
    x = cases.inputs(c)
    monkeypatch.setenv("TRPO_RITZ_RERUN", "0")     # the fp32 solve itself (th0 would be re-solved in fp64)

    def run():
        with _ctx(x) as ctx:
            a = ctx.cg(x["vin"], c["maxiter"], c["resth"])
            b = ctx.cg(x["vin"], c["maxiter"], c["resth"])     # a second solve: K_0 rewrites the cache
            return a, b, ctx.cg_history()[0]

    (g1, g2, gh), (r1, r2, rh) = _both(monkeypatch, run)
    np.testing.assert_array_equal(g1, r1)
    np.testing.assert_array_equal(g2, r1)
    np.testing.assert_array_equal(gh, rh)


@pytest.mark.parametrize("acf", ["lttt", "ltts", "lsso"])
def test_output_activation_needing_y(acf, monkeypatch):
    """act3 = tanh / logistic: y3 is cached too; the runtime-activation kernel variants."""
    L = [15, 16, 16, 3]
    th, obs = synth.make_theta(L), synth.make_obs(1500, 15)
    std = np.array([0.7, 1.0, 1.4])
    v = synth.make_v(synth.num_params(L))

    def run():
        with trpo_amd.Context(L, acf, th, obs, std, 0.1) as ctx:
            return [ctx.fvp(v) for _ in range(2)]

    got, ref = _both(monkeypatch, run)
    np.testing.assert_array_equal(got[0], ref[0])
    np.testing.assert_array_equal(got[1], ref[0])
    zr, _ = oracle.fvp(L, acf, th, obs, std, v)
    assert cases.rel_l2(got[1], zr) <= FVP_TOL


def test_wide_tile_kernel(monkeypatch):
    """2x64 on the one-wave-per-tile kernel (TRPO_COOP=0): T1 = T2 = 4 cached tiles per lane."""
    monkeypatch.setenv("TRPO_COOP", "0")
    c = cases.case("syn_2x64_fvp_n4096")
    x = cases.inputs(c)

    def run():
        with _ctx(x) as ctx:
            assert "coop" not in ctx.kernel_name
            return [ctx.fvp(x["vin"]) for _ in range(2)]

    got, ref = _both(monkeypatch, run)
    np.testing.assert_array_equal(got[1], ref[0])
    assert cases.rel_l2(got[1], cases.expected(c)) <= FVP_TOL


def test_cache_invalidated_by_theta_and_obs():
    """set_theta / set_obs between FVPs: the next FVP must see the new forward pass."""
    L = [15, 16, 16, 3]
    P = synth.num_params(L)
    th1, obs1 = synth.make_theta(L), synth.make_obs(2000, 15)
    rng = np.random.default_rng(7)
    th2 = th1 + 0.05 * rng.standard_normal(P)
    obs2 = obs1[::-1].copy() * 1.3
    std = np.ones(3)
    v = synth.make_v(P)
    with trpo_amd.Context(L, "lttl", th1, obs1, std, 0.1) as ctx:
        ctx.fvp(v)
        ctx.fvp(v)
        ctx.set_theta(th2)
        z2 = ctx.fvp(v)
        ctx.set_obs(obs2)
        z3 = ctx.fvp(v)
        b = synth.make_b(P)
        x3 = ctx.cg(b, 10, 0.0)
    with trpo_amd.Context(L, "lttl", th2, obs1, std, 0.1) as fresh:
        np.testing.assert_array_equal(z2, fresh.fvp(v))
    with trpo_amd.Context(L, "lttl", th2, obs2, std, 0.1) as fresh:
        np.testing.assert_array_equal(z3, fresh.fvp(v))
        np.testing.assert_array_equal(x3, fresh.cg(b, 10, 0.0))
    zr, _ = oracle.fvp(L, "lttl", th2, obs2, std, v)
    assert cases.rel_l2(z3, zr) <= FVP_TOL


@pytest.mark.parametrize("layers,fused", [([15, 16, 16, 3], "1"), ([15, 64, 64, 3], "1"), ([15, 64, 64, 3], "0")])
def test_update_without_cache_writing_cg_leaves_cache_invalid(layers, fused, monkeypatch):
    """set_theta -> update: FVP(x) and every later FVP may read the forward cache only if the
    update's CG actually rewrote it (its fused K_0).  update(max_iter=0) enqueues no FVP in the CG,
    and the unfused cooperative path (TRPO_COOP_FUSED=0) never writes the cache: in both cases the
    next FVP must recompute the forward pass of the NEW theta."""
    monkeypatch.setenv("TRPO_COOP_FUSED", fused)
    P = synth.num_params(layers)
    th1, obs = synth.make_theta(layers), synth.make_obs(2000, layers[0])
    th2 = th1 + 0.05 * np.random.default_rng(11).standard_normal(P)
    th2[-layers[-1]:] = th1[-layers[-1]:]
    std = np.ones(layers[-1])
    v = synth.make_v(P)
    mean, action, adv = synth.make_rollout(layers, "lttl", th2, obs, std)
    zr, _ = oracle.fvp(layers, "lttl", th2, obs, std, v)
    for max_iter in ((0, 10) if fused == "1" else (10,)):
        with trpo_amd.Context(layers, "lttl", th1, obs, std, 0.1) as ctx:
            ctx.fvp(v)                                  # cache now holds th1's activations
            ctx.set_theta(th2)
            ctx.set_rollout(mean, action, adv)
            r = ctx.update(max_iter=max_iter)
            assert r["cg_iters"] <= max_iter and (max_iter > 0 or r["cg_iters"] == 0)
            assert cases.rel_l2(ctx.fvp(v), zr) <= FVP_TOL, max_iter


@pytest.mark.parametrize("layers,acf,n", [([15, 64, 64, 3], "lttl", 4096), ([15, 32, 32, 3], "lttl", 3000),
                                          ([15, 64, 64, 3], "lsso", 2000), ([15, 64, 64, 3], "lttt", 2000),
                                          ([20, 64, 64, 3], "lttl", 1000)])
def test_cooperative_kernel_cache(layers, acf, n, monkeypatch):
    """The fp32 cooperative kernel (wide hidden layers) on the cache: MODE 3 (standalone FVP) and
    MODE 4 (CG iteration) bit-identical to the recomputing kernel; tanh output (y3 needed) and the
    T0 = 2, TH = 4 shape run without the cache and must be unaffected."""
    P = synth.num_params(layers)
    th, obs = synth.make_theta(layers), synth.make_obs(n, layers[0])
    std = np.array([0.7, 1.0, 1.4])
    v, b = synth.make_v(P), synth.make_b(P)

    def run():
        with trpo_amd.Context(layers, acf, th, obs, std, 0.1) as ctx:
            assert "coop" in ctx.kernel_name
            return [ctx.fvp(v), ctx.fvp(v), ctx.cg(b, 10, 0.0), ctx.cg(b, 10, 0.0)]

    got, ref = _both(monkeypatch, run)
    for a, r in zip(got, ref):
        np.testing.assert_array_equal(a, r)
    zr, _ = oracle.fvp(layers, acf, th, obs, std, v)
    assert cases.rel_l2(got[1], zr) <= FVP_TOL
