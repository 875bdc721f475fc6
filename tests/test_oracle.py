"""Pin the CPU oracle (oracle/trpo_oracle.c) to the reference.

The goldens were produced by the reference's own TRPO_FVP.c / TRPO_CG.c /
TRPO_Update.c (tests/golden/make_goldens.py); ArmTestCG.txt is the reference's fixture.
"""
import numpy as np
import pytest

import cases
import oracle

FVPCG = [c for c in cases.manifest() if c["kind"] in ("fvp", "cg")]
FAST = [c["name"] for c in FVPCG if c["n"] <= 5000]
SLOW = [c["name"] for c in FVPCG if c["n"] > 5000]
UPDATE = [c["name"] for c in cases.manifest() if c["kind"] == "update"]
BASELINE = [c["name"] for c in cases.manifest() if c["kind"] == "baseline"]


def _run(c, threads=1):
    x = cases.inputs(c)
    if c["kind"] == "fvp":
        out, _ = oracle.fvp(x["layers"], x["acfunc"], x["theta"], x["obs"], x["std"], x["vin"], x["damping"],
                            threads)
        return out, None
    r = oracle.cg(x["layers"], x["acfunc"], x["theta"], x["obs"], x["std"], x["vin"], c["maxiter"], c["resth"],
                  x["damping"], threads)
    return r["x"], r


@pytest.mark.parametrize("name", FAST)
def test_oracle_matches_reference_golden(name):
    c = cases.case(name)
    out, r = _run(c)
    assert cases.rel_l2(out, cases.expected(c)) <= 1e-12
    if r is not None:
        assert r["iters"] == c["iters"]
        np.testing.assert_allclose(r["rdotr"], c["rdotr"], rtol=1e-10)
        np.testing.assert_allclose(r["xnorm"][1:], c["xnorm"][1:], rtol=1e-10)


@pytest.mark.slow
@pytest.mark.parametrize("name", SLOW)
def test_oracle_matches_reference_golden_50k(name):
    c = cases.case(name)
    out, r = _run(c, threads=4)     # threaded split: only the summation order differs
    assert cases.rel_l2(out, cases.expected(c)) <= 1e-10


def test_oracle_vs_fixture_cg():
    """ArmTestCG.txt column 2 is reproducible at N=3150: relL2 ~8e-6."""
    c = cases.case("fix_cg_n3150_th1e-10")
    out, r = _run(c)
    fx = np.loadtxt(cases.GOLDEN + "/ArmTestCG.txt")[:, 1]
    assert cases.rel_l2(out, fx) < 2e-5
    assert r["iters"] == 8


def test_oracle_forward_matches_fixture_mean():
    """ArmTestData.txt's Mean column equals the policy forward pass."""
    t = np.loadtxt(cases.GOLDEN + "/ArmTestData.txt")
    mean = oracle.forward(cases.ARM, "lttl", cases.fixture_model(), t[:, 6:21])
    rel = np.abs(mean - t[:, 0:3]) / np.abs(t[:, 0:3])
    assert (rel > 0.01).sum() == 0


def test_oracle_threaded_close():
    c = cases.case("fix_fvp_n3150")
    a, _ = _run(c, 1)
    b, _ = _run(c, 3)
    assert cases.rel_l2(a, b) < 1e-13


def _update(c):
    x = cases.update_inputs(c)
    return x, oracle.update(x["layers"], x["acfunc"], x["theta"], x["obs"], x["mean"], x["action"], x["adv"],
                            x["std"], x["damping"])


@pytest.mark.parametrize("name", UPDATE)
def test_oracle_update_matches_reference_golden(name):
    """TRPO_Update restated (policy gradient, CG, step size, line search) vs the reference."""
    c = cases.case(name)
    x, r = _update(c)
    exp = cases.expected(c)
    assert cases.rel_l2(r["theta"], exp) <= 1e-12
    assert r["accepted"] == c["accepted"]
    assert r["evaluated"] == len(c["ratio"])
    np.testing.assert_allclose(r["ratio"], c["ratio"], rtol=1e-9)
    for key in ("shs", "lagrange", "gnorm"):
        assert abs(r[key] - c[key]) <= 1e-11 * abs(c[key]) + 1e-14, key
    assert abs(r["fval"] - c["fval"]) <= 1e-12
    if c["accepted"] < 0:            # reference quirk: theta = the CG step direction
        np.testing.assert_array_equal(r["theta"], r["x"])


def test_oracle_update_fixture_matches_survey_g5():
    """shs 0.00294934722, lagrange 0.543078928, first backtrack accepted, ratio 0.91297."""
    c = cases.case("fix_update_n3150")
    _, r = _update(c)
    assert abs(r["shs"] - 0.00294934722115) < 1e-12
    assert abs(r["lagrange"] - 0.54307892807127) < 1e-10
    assert r["accepted"] == 0 and abs(r["ratio"][0] - 0.91297) < 1e-5


def test_oracle_policy_gradient_is_the_fixture_cg_rhs():
    """ArmTestCG.txt column 1 is TRPO_Update's policy gradient b at N=3150."""
    c = cases.case("fix_update_n3150")
    x = cases.update_inputs(c)
    b, _ = oracle.policy_grad(x["layers"], x["acfunc"], x["theta"], x["obs"], x["mean"], x["action"], x["adv"])
    b_fix = np.loadtxt(cases.GOLDEN + "/ArmTestCG.txt")[:, 0]
    assert cases.rel_l2(b, b_fix) < 1e-6


@pytest.mark.parametrize("name", BASELINE)
def test_oracle_baseline_evaluate_matches_reference(name):
    """evaluate() restated (src/TRPO_Baseline.c:29-240) vs the reference's own evaluate."""
    c = cases.case(name)
    x, obs, tgt = cases.baseline_inputs(c)
    f, g, pred = oracle.baseline_evaluate(c["layers"], c["acfunc"], x, obs, tgt, c["num_ep"], c["ep_len"])
    exp = cases.expected(c)
    assert abs(f - c["f"]) <= 1e-14 * abs(c["f"])
    np.testing.assert_array_equal(g, exp[:c["padded"]])
    np.testing.assert_array_equal(pred, exp[c["padded"]:])
