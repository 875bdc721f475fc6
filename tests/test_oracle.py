"""Pin the CPU oracle (oracle/trpo_oracle.c) to the reference.

The goldens were produced by the reference's own TRPO_FVP.c / TRPO_CG.c
(tests/golden/make_goldens.py); ArmTestCG.txt is the reference's fixture.
"""
import numpy as np
import pytest

import cases
import oracle

FAST = [c["name"] for c in cases.manifest() if c["n"] <= 5000]
SLOW = [c["name"] for c in cases.manifest() if c["n"] > 5000]


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
