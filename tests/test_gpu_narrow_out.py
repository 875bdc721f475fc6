"""MI355X: the narrow output layer of the small-net tile kernel (fvp_mlp3_kernel NO > 0).

For policies with at most 4 outputs the output layer's forward / R-forward run on
v_mfma_f32_4x4x1_16b_f32 and G2 = W2 G3 on the VALU; its two twins differ in the RGW2 / B3
contraction -- on the 16x16x4 MFMA ("no-mfma", few tiles per wave) or as per-lane VALU partials
("no-valu", many tiles per wave) -- and set_obs picks one by tiles per wave
(TRPO_NO_VALU_MIN_TILES, default 4).  TRPO_NARROW_OUT=0 keeps the 16x16x4 output layer.
Also the cooperative kernel's narrow output layer (wide hidden layers: no4 coop).
Checked: both twins against the oracle (FVP, CG, policy gradient, full update) for 1..4 outputs and
every output activation, the forward cache bit for bit against recomputing for both twins, agreement
with the 16x16x4 output layer to fp32 rounding, the per-N choice, and that a context re-binds its twin
when set_obs changes N (the CG graph recaptured, the y cache invalidated).
"""
import numpy as np
import pytest

import cases
import oracle
import trpo_amd
from trpo_amd import synth

pytestmark = pytest.mark.gpu

FVP_TOL, CG_TOL = 1e-5, 1e-4
TWINS = {"no-mfma": "1000000", "no-valu": "0"}       # TRPO_NO_VALU_MIN_TILES forcing each twin


def _problem(L, acts, n, seed=7):
    th, obs = synth.make_theta(L, seed=seed), synth.make_obs(n, L[0], seed=seed + 1)
    std = np.linspace(0.7, 1.3, L[-1])
    P = synth.num_params(L)
    return th, obs, std, synth.make_v(P, seed=seed + 2), synth.make_b(P, seed=seed + 3)


@pytest.mark.parametrize("twin", list(TWINS))
@pytest.mark.parametrize("L,acts", [([15, 16, 16, 3], "lttl"), ([15, 16, 16, 1], "lttl"), ([12, 9, 14, 2], "lstt"),
                                    ([16, 16, 16, 4], "lots"), ([15, 16, 16, 3], "ltts")])
def test_twins_against_oracle(L, acts, twin, monkeypatch):
    monkeypatch.setenv("TRPO_NO_VALU_MIN_TILES", TWINS[twin])
    n = 2777
    th, obs, std, v, b = _problem(L, acts, n)
    zr, _ = oracle.fvp(L, acts, th, obs, std, v)
    xr = oracle.cg(L, acts, th, obs, std, b, 10, 0.0)["x"]
    mean, action, adv = synth.make_rollout(L, acts, th, obs, std)
    ref = oracle.update(L, acts, th, obs, mean, action, adv, std, 0.1)
    bref, _ = oracle.policy_grad(L, acts, th, obs, mean, action, adv)
    with trpo_amd.Context(L, acts, th, obs, std, 0.1) as ctx:
        assert ctx.kernel_name.endswith(twin), ctx.kernel_name
        z1, z2 = ctx.fvp(v), ctx.fvp(v)                 # recompute (writes the cache), then cached
        x = ctx.cg(b, 10, 0.0)
        ctx.set_rollout(mean, action, adv)
        r = ctx.update()
    np.testing.assert_array_equal(z1, z2)
    assert cases.rel_l2(z1, zr) <= FVP_TOL
    assert cases.rel_l2(x, xr) <= CG_TOL
    assert cases.rel_l2(r["b"], bref) <= 2e-6
    assert r["accepted"] == ref["accepted"]
    assert cases.rel_l2(r["x"], ref["x"]) <= CG_TOL


@pytest.mark.parametrize("twin", list(TWINS))
@pytest.mark.parametrize("name", ["fix_cg_n3150_th0", "syn_sigma_cg", "syn_arm_cg_n50000"])
def test_twins_cache_bitwise_and_golden(name, twin, monkeypatch):
    """Each twin on the forward cache gives the bits of the same twin recomputing (TRPO_YCACHE=0)."""
    monkeypatch.setenv("TRPO_NO_VALU_MIN_TILES", TWINS[twin])
    c = cases.case(name)
    x = cases.inputs(c)

    def run():
        with trpo_amd.Context(x["layers"], x["acfunc"], x["theta"], x["obs"], x["std"], x["damping"]) as ctx:
            assert ctx.kernel_name.endswith(twin), ctx.kernel_name
            return ctx.cg(x["vin"], c["maxiter"], c["resth"]), ctx.fvp(x["vin"])

    monkeypatch.setenv("TRPO_YCACHE", "0")
    xr, zr = run()
    monkeypatch.delenv("TRPO_YCACHE")
    xg, zg = run()
    np.testing.assert_array_equal(xg, xr)
    np.testing.assert_array_equal(zg, zr)
    assert cases.rel_l2(xg, cases.expected(c)) <= CG_TOL


def test_narrow_matches_16x16_output_layer(monkeypatch):
    """Same problem with TRPO_NARROW_OUT=0: FVP to fp32 rounding, CG step well inside the bound."""
    c = cases.case("syn_arm_cg_n50000")
    x = cases.inputs(c)
    out = {}
    for no in ("1", "0"):
        monkeypatch.setenv("TRPO_NARROW_OUT", no)
        with trpo_amd.Context(x["layers"], x["acfunc"], x["theta"], x["obs"], x["std"], x["damping"]) as ctx:
            out[no] = (ctx.kernel_name, ctx.fvp(x["vin"]), ctx.cg(x["vin"], 10, 0.0))
    assert "no-" in out["1"][0] and "no-" not in out["0"][0]
    assert cases.rel_l2(out["1"][1], out["0"][1]) <= 1e-6
    assert cases.rel_l2(out["1"][2], out["0"][2]) <= 1e-5


def test_twin_follows_n_and_rebinds(monkeypatch):
    """Default choice by tiles per wave (256 blocks x 8 waves): 50k -> MFMA RGW2, 500k -> VALU RGW2; a
    context whose set_obs changes N re-binds its twin and still solves correctly."""
    monkeypatch.delenv("TRPO_NO_VALU_MIN_TILES", raising=False)
    L = [15, 16, 16, 3]
    th, small, std, v, b = _problem(L, "lttl", 50000)
    big = synth.make_obs(500000, 15, seed=99)
    with trpo_amd.Context(L, "lttl", th, small, std, 0.1) as ctx:
        assert ctx.kernel_name.endswith("no-mfma"), ctx.kernel_name
        x_small = ctx.cg(b, 10, 0.0)
        ctx.set_obs(big)
        assert ctx.kernel_name.endswith("no-valu"), ctx.kernel_name
        x_big = ctx.cg(b, 10, 0.0)
        z_big = ctx.fvp(v)
        ctx.set_obs(small)
        assert ctx.kernel_name.endswith("no-mfma"), ctx.kernel_name
        np.testing.assert_array_equal(ctx.cg(b, 10, 0.0), x_small)
    assert cases.rel_l2(x_small, oracle.cg(L, "lttl", th, small, std, b, 10, 0.0)["x"]) <= CG_TOL
    zr, _ = oracle.fvp(L, "lttl", th, big, std, v)
    assert cases.rel_l2(z_big, zr) <= FVP_TOL
    assert np.all(np.isfinite(x_big))


@pytest.mark.parametrize("L,acts", [([15, 64, 64, 3], "lttl"), ([20, 32, 32, 4], "lstl"), ([30, 48, 48, 2], "ltol"),
                                    ([15, 64, 64, 3], "ltts")])
def test_cooperative_kernel_narrow_output(L, acts, monkeypatch):
    """The cooperative kernel's narrow output layer ("no4 coop", fp32, <= 4 outputs): FVP / CG / update
    against the oracle, the forward cache bit for bit against recomputing, and the 16x16x4 output layer
    (TRPO_NARROW_OUT=0) to fp32 rounding."""
    n = 3001
    th, obs, std, v, b = _problem(L, acts, n, seed=11)
    zr, _ = oracle.fvp(L, acts, th, obs, std, v)
    xr = oracle.cg(L, acts, th, obs, std, b, 10, 0.0)["x"]
    mean, action, adv = synth.make_rollout(L, acts, th, obs, std)
    ref = oracle.update(L, acts, th, obs, mean, action, adv, std, 0.1)

    def run():
        with trpo_amd.Context(L, acts, th, obs, std, 0.1) as ctx:
            name = ctx.kernel_name
            z1, z2 = ctx.fvp(v), ctx.fvp(v)
            x = ctx.cg(b, 10, 0.0)
            ctx.set_rollout(mean, action, adv)
            return name, z1, z2, x, ctx.update()

    name, z1, z2, x, r = run()
    assert name.endswith("no4 coop"), name
    np.testing.assert_array_equal(z1, z2)
    assert cases.rel_l2(z1, zr) <= FVP_TOL
    assert cases.rel_l2(x, xr) <= CG_TOL
    assert r["accepted"] == ref["accepted"]
    assert cases.rel_l2(r["x"], ref["x"]) <= CG_TOL
    monkeypatch.setenv("TRPO_YCACHE", "0")
    _, z0, _, x0, _ = run()
    np.testing.assert_array_equal(z0, z1)
    np.testing.assert_array_equal(x0, x)
    monkeypatch.setenv("TRPO_NARROW_OUT", "0")
    name16, z16, _, x16, _ = run()
    assert "no4" not in name16
    assert cases.rel_l2(z16, z1) <= 1e-6
    assert cases.rel_l2(x16, x) <= 1e-5
