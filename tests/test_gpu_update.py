"""MI355X parity of the TRPO_Update path (src/TRPO_Update.c:10-1011) through the C ABI.

Tolerances (stated):
  * policy gradient b: weights/biases by the fp32 MFMA tile kernel (fp64 cross-tile sums),
    LogStd part and sum(Adv) in fp64 -> relL2 <= 2e-6 (numpy emulation of fp32 per-sample math:
    1.2e-7, which moves the CG step by 4e-7); the generic fp64 kernel (TRPO_UPDATE_GENERIC=1,
    used for shapes without a tile kernel) -> relL2 <= 1e-12
  * CG step x: fp32 FVP inside the solve -> relL2 <= 1e-4 (as the CG tests) for every case, the
    2x64 policy included.  Without the device CG's residual reorthogonalisation the
    fp32 rounding of each CG direction p (and the p-proportional rounding of the R chains) is noise
    that CG amplifies by the condition number: 7.7e-4 on the 2x64 case (numpy emulation of fp32
    per-sample math: 7.6e-4; with reorthogonalisation 8e-8, tools/cg_noise_variants.py).
  * step size shs / lagrange: derived from x -> rel <= 1e-4
  * parameter update theta' - theta: relL2 <= 1e-4 against the reference's own TRPO_Update
  * line search: same accepted backtrack as the reference, ratios within rtol 1e-3
"""
import os

import numpy as np
import pytest

import cases
import trpo_amd

pytestmark = pytest.mark.gpu

UPDATE = [c["name"] for c in cases.manifest() if c["kind"] == "update"]
TOL = {}
B_TOL = 2e-6            # fp32 tile-kernel policy gradient
B_TOL_GENERIC = 1e-12   # fp64 generic kernel


def _ctx(x):
    ctx = trpo_amd.Context(x["layers"], x["acfunc"], x["theta"], x["obs"], x["std"], x["damping"])
    ctx.set_rollout(x["mean"], x["action"], x["adv"])
    return ctx


def _oracle_update(x, **kw):
    import oracle
    return oracle.update(x["layers"], x["acfunc"], x["theta"], x["obs"], x["mean"], x["action"], x["adv"],
                         x["std"], x["damping"], **kw)


@pytest.mark.parametrize("generic", [False, True])
@pytest.mark.parametrize("name", UPDATE)
def test_update_matches_reference_golden(name, generic, monkeypatch):
    import oracle
    if generic:
        monkeypatch.setenv("TRPO_UPDATE_GENERIC", "1")
    c = cases.case(name)
    x = cases.update_inputs(c)
    with _ctx(x) as ctx:
        r = ctx.update()
    b_ref, _ = oracle.policy_grad(x["layers"], x["acfunc"], x["theta"], x["obs"], x["mean"], x["action"], x["adv"])
    assert cases.rel_l2(r["b"], b_ref) <= (B_TOL_GENERIC if generic else B_TOL)
    assert abs(r["gnorm"] - c["gnorm"]) <= (B_TOL_GENERIC if generic else B_TOL) * c["gnorm"]
    assert abs(r["fval"] - c["fval"]) <= 1e-12
    tol = TOL.get(name, 1e-4)
    ref = _oracle_update(x)
    assert cases.rel_l2(r["x"], ref["x"]) <= tol
    assert abs(r["shs"] - c["shs"]) <= tol * abs(c["shs"])
    assert abs(r["lagrange"] - c["lagrange"]) <= tol * abs(c["lagrange"])
    assert r["accepted"] == c["accepted"]
    assert r["evaluated"] == len(c["ratio"])
    np.testing.assert_allclose(r["ratio"], c["ratio"], rtol=1e-3)
    exp = cases.expected(c)
    if c["accepted"] >= 0:
        assert cases.rel_l2(r["theta"] - x["theta"], exp - x["theta"]) <= tol
    else:                                   # reference quirk: the CG step direction is returned
        np.testing.assert_array_equal(r["theta"], r["x"])
        assert cases.rel_l2(r["theta"], exp) <= tol


def test_trpo_update_file_entry_point(capfd):
    """TRPOCpuCode.c-style call (src/TRPOCpuCode.c:314-360) on the reference fixtures."""
    trpo_amd.cache_clear()
    g = cases.GOLDEN
    prm = trpo_amd.make_param(os.path.join(g, "ArmTestModel.txt"), os.path.join(g, "ArmTestData.txt"),
                              [15, 16, 16, 3], "lttl", 3150, 0.1)
    res = np.zeros(582)
    assert trpo_amd.TRPO_Update(prm, res, 6) >= 0
    c = cases.case("fix_update_n3150")
    th = cases.fixture_model()
    assert cases.rel_l2(res - th, cases.expected(c) - th) <= 1e-4
    out = capfd.readouterr().out
    assert out.count("CG Iter[") == 9                  # 8 FVPs, as the reference (reorthogonalised CG)
    import re
    shs = float(re.search(r"shs: (\S+)", out).group(1))
    lm, gn = map(float, re.search(r"lagrange multiplier: (\S+), gnorm: (\S+)", out).groups())
    are = re.findall(r"a/e/r (\S+) / (\S+) / (\S+)", out)
    assert abs(shs - c["shs"]) <= 1e-4 * c["shs"] and abs(lm - c["lagrange"]) <= 1e-4 * c["lagrange"]
    assert abs(gn - c["gnorm"]) <= B_TOL * c["gnorm"]
    assert len(are) == 1 and abs(float(are[0][2]) - c["ratio"][0]) <= 1e-3 * c["ratio"][0]
    # a second call hits the device cache (rollout already resident): same answer
    res2 = np.zeros(582)
    assert trpo_amd.TRPO_Update(prm, res2, 1) >= 0
    np.testing.assert_array_equal(res, res2)


def test_update_later_backtrack_accepted():
    """max_kl = 20: the first two step fractions are rejected, the third accepted -- exercises the
    batched evaluation of the remaining fractions (one launch) against the sequential oracle."""
    from trpo_amd import synth
    L = [15, 16, 16, 3]
    th = synth.make_theta(L)
    obs = synth.make_obs(3000, 15)
    std = np.ones(3)
    mean, action, adv = synth.make_rollout(L, "lttl", th, obs, std)
    x = dict(layers=L, acfunc="lttl", theta=th, obs=obs, std=std, mean=mean, action=action, adv=adv, damping=0.1)
    ref = _oracle_update(x, max_kl=20.0)
    assert ref["accepted"] == 2
    with _ctx(x) as ctx:
        r = ctx.update(max_kl=20.0)
    assert r["accepted"] == 2 and r["evaluated"] == 3
    np.testing.assert_allclose(r["ratio"], ref["ratio"], rtol=1e-3, atol=1e-6)
    assert cases.rel_l2(r["theta"] - th, ref["theta"] - th) <= 1e-4


@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000])
def test_update_ragged_sample_counts(n):
    import oracle
    from trpo_amd import synth
    L = [15, 64, 64, 3]
    th = synth.make_theta(L)
    obs = synth.make_obs(n, 15)
    std = np.array([0.6065306597126334, 1.0, 1.2840254166877414])
    th[-3:] = [-0.5, 0.0, 0.25]
    mean, action, adv = synth.make_rollout(L, "lttl", th, obs, std)
    x = dict(layers=L, acfunc="lttl", theta=th, obs=obs, std=std, mean=mean, action=action, adv=adv, damping=0.1)
    b_ref, s_ref = oracle.policy_grad(L, "lttl", th, obs, mean, action, adv)
    with _ctx(x) as ctx:
        r = ctx.update()
    assert cases.rel_l2(r["b"], b_ref) <= B_TOL
    assert abs(r["fval"] + s_ref / n) <= 1e-12 * max(1.0, abs(s_ref / n))


def test_update_requires_rollout():
    c = cases.case("fix_update_n3150")
    x = cases.update_inputs(c)
    with trpo_amd.Context(x["layers"], x["acfunc"], x["theta"], x["obs"], x["std"]) as ctx:
        with pytest.raises(trpo_amd.TRPOError):
            ctx.update()
        ctx.set_rollout(x["mean"], x["action"], x["adv"])
        ctx.update()
        ctx.set_obs(x["obs"][:100])                   # new samples invalidate the rollout
        with pytest.raises(trpo_amd.TRPOError):
            ctx.update()


@pytest.mark.parametrize("layers", [[15, 16, 16, 3], [15, 64, 64, 3]])
def test_repeated_updates_deterministic(layers, monkeypatch):
    """A trainer-like sequence on one context -- several updates, set_theta / set_rollout between them,
    a rejected full step, each update repeated -- is deterministic: a run with every CG launched
    eagerly (TRPO_NO_GRAPH=1) and a run on the captured, replayed CG graphs agree bit for bit (the
    device state the update reuses across calls: forward cache, replica sets, rollout rows, graphs).  Eager
    is the default launch form since round 4 (TRPO_CG_GRAPH=1 selects the graph)."""
    from trpo_amd import synth
    n = 3000
    th0, obs = synth.make_theta(layers), synth.make_obs(n, layers[0])
    std = np.ones(layers[-1])

    def run():
        out = []
        th = th0.copy()
        with trpo_amd.Context(layers, "lttl", th, obs, std, 0.1) as ctx:
            for it in range(4):
                mean, action, adv = synth.make_rollout(layers, "lttl", th, obs, std)
                if it == 3:
                    adv = -adv              # sign-flipped advantages: the full step is rejected
                ctx.set_rollout(mean, action, adv)
                r = ctx.update()
                r2 = ctx.update()          # same rollout and theta: the replayed graph
                out.append((r["theta"], r["x"], r["b"], r2["theta"], r2["ratio"], r["accepted"], r2["accepted"]))
                th = r["theta"]
                ctx.set_theta(th)
        return out

    monkeypatch.setenv("TRPO_NO_GRAPH", "1")         # read by the library at every CG enqueue
    eager = run()
    monkeypatch.delenv("TRPO_NO_GRAPH")
    monkeypatch.setenv("TRPO_CG_GRAPH", "1")
    graph = run()
    monkeypatch.delenv("TRPO_CG_GRAPH")
    for a, e in zip(graph, eager):
        for x, y in zip(a, e):
            np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("solves", ["update", "enqueue_cg"])
def test_fvp_of_v_after_replayed_solves(solves, monkeypatch):
    """the cooperative kernel's direction pack holds V after an upload, and every CG
    solve overwrites it with its directions -- also a solve replayed from the captured graph, whose
    host-side enqueue ran only at capture.  Sequence: upload V, two graph-mode solves (the update path's
    CG is always the replayed graph; enqueue_cg with TRPO_CG_GRAPH=1), then an FVP of slot V: it must be
    F v, not F of the last CG direction."""
    from trpo_amd import synth
    layers, n = [15, 64, 64, 3], 3000                   # 2x64: the cooperative kernel (pre-packed direction)
    th, obs = synth.make_theta(layers), synth.make_obs(n, layers[0])
    std = np.ones(layers[-1])
    v = synth.make_v(synth.num_params(layers))
    if solves == "enqueue_cg":
        monkeypatch.setenv("TRPO_CG_GRAPH", "1")
    with trpo_amd.Context(layers, "lttl", th, obs, std, 0.1) as ctx:
        z_ref = ctx.fvp(v)
        mean, action, adv = synth.make_rollout(layers, "lttl", th, obs, std)
        ctx.set_rollout(mean, action, adv)
        ctx.upload_b(synth.make_b(synth.num_params(layers)))
        ctx.upload_v(v)
        for _ in range(2):
            if solves == "update":
                ctx.update()
            else:
                ctx.enqueue_cg(10, 0.0)
        ctx.enqueue_fvp()
        ctx.synchronize()
        z = ctx.download_z()
    assert cases.rel_l2(z, z_ref) <= 1e-6


def test_updates_with_changing_max_iter():
    """Round 6: an update's results come back through pinned memory behind per-block flag words whose
    offset moves with max_iter (the history's length).  Updates on one context with max_iter 10, 4, 12, 10
    each equal the same update on a fresh context, bit for bit."""
    from trpo_amd import synth
    layers, n = [15, 16, 16, 3], 3000
    th, obs = synth.make_theta(layers), synth.make_obs(n, layers[0])
    std = np.ones(layers[-1])
    mean, action, adv = synth.make_rollout(layers, "lttl", th, obs, std)
    with trpo_amd.Context(layers, "lttl", th, obs, std, 0.1) as ctx:
        ctx.set_rollout(mean, action, adv)
        got = [(m, ctx.update(max_iter=m)) for m in (10, 4, 12, 10)]
    for m, r in got:
        with trpo_amd.Context(layers, "lttl", th, obs, std, 0.1) as fresh:
            fresh.set_rollout(mean, action, adv)
            f = fresh.update(max_iter=m)
        for key in ("theta", "x", "b"):
            np.testing.assert_array_equal(r[key], f[key], err_msg="max_iter %d %s" % (m, key))
        assert r["accepted"] == f["accepted"] and r["shs"] == f["shs"]
