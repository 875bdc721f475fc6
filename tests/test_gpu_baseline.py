"""MI355X parity of the value-baseline objective (src/TRPO_Baseline.c:29-240).

The device computes in fp64 (one sample per lane), only the summation order differs from the
reference, so: objective rel <= 1e-13, gradient and predictions relL2 <= 1e-12.  A full L-BFGS
fit (scipy's L-BFGS-B driving the device objective vs the same driver on the oracle) ends on
the same parameters to 1e-8.
"""
import numpy as np
import pytest

import cases
import trpo_amd

pytestmark = pytest.mark.gpu

BASELINE = [c["name"] for c in cases.manifest() if c["kind"] == "baseline"]


@pytest.mark.parametrize("name", BASELINE)
def test_baseline_context_matches_reference(name):
    c = cases.case(name)
    x, obs, tgt = cases.baseline_inputs(c)
    exp = cases.expected(c)
    with trpo_amd.Baseline(c["layers"], c["acfunc"]) as b:
        b.set_data(obs, tgt, c["num_ep"], c["ep_len"])
        f, g, pred = b.evaluate(x, want_predict=True)
    assert abs(f - c["f"]) <= 1e-13 * abs(c["f"])
    assert cases.rel_l2(g, exp[:c["padded"]]) <= 1e-12
    assert np.all(g[b.np:] == 0.0)
    assert cases.rel_l2(pred, exp[c["padded"]:]) <= 1e-12


@pytest.mark.parametrize("name", BASELINE)
def test_lane_kernel_matches_one_lane_kernel(name, monkeypatch):
    """The lane-parallel kernel (round 5, [L0, L1, L2, 1] nets with widths <= 16) keeps every per-sample
    value's bits (predictions identical) and changes only the order of the sums over samples; the one-lane
    kernel (TRPO_BASELINE_LANE=0, read at set_data) stays the path for every other shape."""
    c = cases.case(name)
    x, obs, tgt = cases.baseline_inputs(c)
    out = {}
    for lane in ("1", "0"):
        monkeypatch.setenv("TRPO_BASELINE_LANE", lane)
        with trpo_amd.Baseline(c["layers"], c["acfunc"]) as b:
            b.set_data(obs, tgt, c["num_ep"], c["ep_len"])
            out[lane] = b.evaluate(x, want_predict=True)
    np.testing.assert_array_equal(out["1"][2], out["0"][2])
    assert abs(out["1"][0] - out["0"][0]) <= 1e-14 * abs(out["0"][0])
    assert cases.rel_l2(out["1"][1], out["0"][1]) <= 1e-13


def test_evaluate_drop_in_callback():
    """lbfgs()-style calls through the exported evaluate(TRPOBaselineParam*, x, g, n, step)."""
    c = cases.case("syn_baseline_n3000")
    x, obs, tgt = cases.baseline_inputs(c)
    exp = cases.expected(c)
    p = trpo_amd.make_baseline_param(c["layers"], c["acfunc"], obs, tgt, c["num_ep"], c["ep_len"])
    g = np.zeros(c["padded"])
    f = trpo_amd.evaluate(p, x, g)
    assert abs(f - c["f"]) <= 1e-13 * abs(c["f"])
    assert cases.rel_l2(g, exp[:c["padded"]]) <= 1e-12
    assert cases.rel_l2(p.predict, exp[c["padded"]:]) <= 1e-12
    np.testing.assert_array_equal(p.W[0], x[:16 * 16])          # W/B left = x, like the reference
    # the caller rewrites its data between fits: the cached upload must notice
    tgt2 = tgt * 0.5 + 1.0
    p2 = trpo_amd.make_baseline_param(c["layers"], c["acfunc"], obs, tgt2, c["num_ep"], c["ep_len"])
    f2 = trpo_amd.evaluate(p2, x, g)
    import oracle
    fr, gr, _ = oracle.baseline_evaluate(c["layers"], c["acfunc"], x, obs, tgt2, c["num_ep"], c["ep_len"])
    assert abs(f2 - fr) <= 1e-13 * abs(fr) and cases.rel_l2(g, gr) <= 1e-12


def test_evaluate_rejects_unsupported_activation():
    x, obs, tgt = trpo_amd.synth.make_baseline_problem([16, 16, 16, 1], 2, 10)
    p = trpo_amd.make_baseline_param([16, 16, 16, 1], "lstl", obs, tgt, 2, 10)
    assert trpo_amd.evaluate(p, x, np.zeros(x.size)) == -1.0


def test_lbfgs_fit_matches_oracle_fit():
    scipy_opt = pytest.importorskip("scipy.optimize")
    import oracle
    L, acf, nep, eplen = [16, 16, 16, 1], "lttl", 20, 150
    x0, obs, tgt = trpo_amd.synth.make_baseline_problem(L, nep, eplen)
    with trpo_amd.Baseline(L, acf) as b:
        b.set_data(obs, tgt, nep, eplen)
        xd, fd, _ = scipy_opt.fmin_l_bfgs_b(lambda v: b.evaluate(v), x0, maxiter=25)
    xo, fo, _ = scipy_opt.fmin_l_bfgs_b(
        lambda v: oracle.baseline_evaluate(L, acf, v, obs, tgt, nep, eplen)[:2], x0, maxiter=25)
    assert fd < 0.9 * oracle.baseline_evaluate(L, acf, x0, obs, tgt, nep, eplen)[0]   # it fits
    assert cases.rel_l2(xd, xo) <= 1e-8
    assert abs(fd - fo) <= 1e-10 * abs(fo)


@pytest.mark.parametrize("num_ep,ep_len", [(1, 20), (5, 106), (20, 150), (40, 300)])
def test_lane_kernel_grids_and_handoff(num_ep, ep_len, monkeypatch):
    """Round 6: the lane kernel takes theta by value and its slab sum hands the result over through pinned
    memory (per-block flag words the host spins on).  Batches giving grids of 2, 34, 188 and 256 blocks
    (one sample per 16-lane group, at most 256 blocks) against the one-lane kernel, and repeated calls --
    with and without predictions, on changing parameters -- bit-identical to a fresh context's."""
    L, acf = [16, 16, 16, 1], "lttl"
    x, obs, tgt = trpo_amd.synth.make_baseline_problem(L, num_ep, ep_len)
    xs = [x, x * 0.9 + 0.01, x]
    monkeypatch.setenv("TRPO_BASELINE_LANE", "0")
    with trpo_amd.Baseline(L, acf) as b:
        b.set_data(obs, tgt, num_ep, ep_len)
        ref = [b.evaluate(v, want_predict=True) for v in xs]
    monkeypatch.setenv("TRPO_BASELINE_LANE", "1")
    with trpo_amd.Baseline(L, acf) as b:
        b.set_data(obs, tgt, num_ep, ep_len)
        got = [b.evaluate(v, want_predict=(k % 2 == 0)) for k in range(6) for v in xs]
    with trpo_amd.Baseline(L, acf) as b:
        b.set_data(obs, tgt, num_ep, ep_len)
        fresh = [b.evaluate(v, want_predict=True) for v in xs]
    for k, r in enumerate(got):
        f = fresh[k % 3]
        assert r[0] == f[0]
        np.testing.assert_array_equal(r[1], f[1])
        if len(r) == 3:
            np.testing.assert_array_equal(r[2], f[2])
    for f, r in zip(fresh, ref):
        np.testing.assert_array_equal(f[2], r[2])
        assert abs(f[0] - r[0]) <= 1e-14 * abs(r[0])
        assert cases.rel_l2(f[1], r[1]) <= 1e-13


def test_evaluate_sees_arrays_rewritten_in_place():
    """Round 6: the drop-in evaluate starts the device on the data it uploaded and compares the caller's
    arrays meanwhile; arrays rewritten IN PLACE (same addresses) between callbacks must still give the
    new data's objective -- the stale result is dropped and the evaluation repeated (observations, then
    targets, then unchanged again)."""
    import oracle
    c = cases.case("syn_baseline_n3000")
    x, obs, tgt = cases.baseline_inputs(c)
    p = trpo_amd.make_baseline_param(c["layers"], c["acfunc"], obs, tgt, c["num_ep"], c["ep_len"])
    o_arr, t_arr = p._keep[0], p._keep[1]
    g = np.zeros(c["padded"])
    trpo_amd.evaluate(p, x, g)
    for change in ("obs", "tgt", None):
        if change == "obs":
            o_arr[7, 3] += 0.25
        elif change == "tgt":
            t_arr[11] -= 0.5
        f = trpo_amd.evaluate(p, x, g)
        fr, gr, pr = oracle.baseline_evaluate(c["layers"], c["acfunc"], x, o_arr, t_arr, c["num_ep"], c["ep_len"])
        assert abs(f - fr) <= 1e-13 * abs(fr), change
        assert cases.rel_l2(g, gr) <= 1e-12, change
        assert cases.rel_l2(p.predict, pr) <= 1e-12, change


def test_evaluate_after_set_data_shrinks():
    """Round 6: the lane path's flag words sit behind the predictions, so they move when set_data changes
    the sample count; evaluations after a larger and then a smaller batch on one context equal a fresh
    context's, bit for bit."""
    L, acf = [16, 16, 16, 1], "lttl"
    big = trpo_amd.synth.make_baseline_problem(L, 20, 150)
    small = trpo_amd.synth.make_baseline_problem(L, 7, 111)
    with trpo_amd.Baseline(L, acf) as b:
        got = []
        for x, obs, tgt, ne, el in ((*big, 20, 150), (*small, 7, 111), (*big, 20, 150)):
            b.set_data(obs, tgt, ne, el)
            got.append((b.evaluate(x, want_predict=True), b.evaluate(x)))
    for (x, obs, tgt, ne, el), (r, r2) in zip(((*big, 20, 150), (*small, 7, 111), (*big, 20, 150)), got):
        with trpo_amd.Baseline(L, acf) as f:
            f.set_data(obs, tgt, ne, el)
            e = f.evaluate(x, want_predict=True)
        assert r[0] == e[0] and r2[0] == e[0]
        np.testing.assert_array_equal(r[1], e[1])
        np.testing.assert_array_equal(r2[1], e[1])
        np.testing.assert_array_equal(r[2], e[2])
