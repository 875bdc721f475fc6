"""The library's multi-rank shard path on ONE GPU (reference CG loop
src/TRPO_CG.c:45-104 around the per-sample FVP loop src/TRPO_FVP.c:771-921).

Two (or three) contexts in one process, each on a contiguous shard of the samples, are joined by the
in-process host group (trpo_ctx_attach_group): the same code path a multi-GPU run takes under RCCL --
the N all-reduce at attach, division by the GLOBAL N, replica sets sized from the LARGEST shard, one
all-reduce of the partial sum per FVP, every rank running the identical CG -- with the collective
done as a host-staged rank-order sum.  Each rank is driven by its own thread (ctypes releases the GIL),
as one process per GPU would be.

Checked: every rank ends with a bit-identical step x (lockstep CG), x is within the north-star bound
of the reference's golden, the replica count is the one the largest shard's grid implies, and the
FVP and the full update agree across ranks.
"""
import threading

import numpy as np
import pytest

import cases
import trpo_amd
from trpo_amd import synth

pytestmark = pytest.mark.gpu

CG_TOL = 1e-4


def _cdiv(a, b):
    return -(-a // b)


def run_ranks(ctxs, fn, timeout=120.0):
    """fn(ctx, rank) on every context concurrently, one thread each, after attaching them to a group."""
    world = len(ctxs)
    group = trpo_amd.Group(world)
    out, err = [None] * world, [None] * world

    def work(r):
        try:
            ctxs[r].attach_group(group, r)
            out[r] = fn(ctxs[r], r)
        except BaseException as e:          # noqa: BLE001 -- reported below
            err[r] = e

    ts = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout)
    assert not any(t.is_alive() for t in ts), "a rank did not finish (group exchange stuck)"
    for e in err:
        if e is not None:
            raise e
    group.close()
    return out


def _shard_ctxs(x, bounds):
    return [trpo_amd.Context(x["layers"], x["acfunc"], x["theta"], x["obs"][lo:hi], x["std"], x["damping"])
            for lo, hi in bounds]


@pytest.mark.parametrize("bounds", [[(0, 25000), (25000, 50000)], [(0, 10000), (10000, 30001), (30001, 50000)]])
def test_sharded_cg_lockstep_and_golden(bounds):
    c = cases.case("syn_arm_cg_n50000")
    x = cases.inputs(c)
    ctxs = _shard_ctxs(x, bounds)
    try:
        res = run_ranks(ctxs, lambda ctx, r: (ctx.cg(x["vin"], c["maxiter"], c["resth"]), ctx.cg_history(),
                                              ctx.comm_info()))
    finally:
        for ctx in ctxs:
            ctx.close()
    x0, (rr0, xn0, it0), info0 = res[0]
    nmax = max(hi - lo for lo, hi in bounds)
    grid = min(_cdiv(_cdiv(nmax, 16), 8), 256)          # the armDOF_0 tile kernel: 8 tiles per block step
    for r, (xr, (rr, xn, it), info) in enumerate(res):
        np.testing.assert_array_equal(xr, x0)            # lockstep: bit-identical on every rank
        np.testing.assert_array_equal(rr, rr0)
        assert it == it0 == c["iters"]
        assert info["rank"] == r and info["world"] == len(bounds)
        assert info["replicas"] == min(6, max(1, _cdiv(grid, 32))), info   # RMAX = 6
    assert cases.rel_l2(x0, cases.expected(c)) <= CG_TOL


def test_sharded_fvp_matches_golden():
    c = cases.case("fix_fvp_n3150")
    x = cases.inputs(c)
    ctxs = _shard_ctxs(x, [(0, 1000), (1000, 3150)])
    try:
        res = run_ranks(ctxs, lambda ctx, r: ctx.fvp(x["vin"]))
    finally:
        for ctx in ctxs:
            ctx.close()
    np.testing.assert_array_equal(res[0], res[1])
    assert cases.rel_l2(res[0], cases.expected(c)) <= 1e-5


@pytest.mark.parametrize("layers", [[15, 16, 16, 3], [15, 64, 64, 3]])
def test_sharded_update_matches_single_context(layers):
    """TRPO_Update on two shards (policy-gradient, FVP and surrogate all-reduces) against the same
    update on one context over all samples."""
    n = 6000
    th, obs = synth.make_theta(layers), synth.make_obs(n, layers[0])
    std = np.ones(layers[-1])
    mean, action, adv = synth.make_rollout(layers, "lttl", th, obs, std)
    with trpo_amd.Context(layers, "lttl", th, obs, std, 0.1) as one:
        one.set_rollout(mean, action, adv)
        ref = one.update()
    bounds = [(0, 2500), (2500, n)]
    ctxs = [trpo_amd.Context(layers, "lttl", th, obs[lo:hi], std, 0.1) for lo, hi in bounds]
    for ctx, (lo, hi) in zip(ctxs, bounds):
        ctx.set_rollout(mean[lo:hi], action[lo:hi], adv[lo:hi])
    try:
        res = run_ranks(ctxs, lambda ctx, r: ctx.update())
    finally:
        for ctx in ctxs:
            ctx.close()
    for key in ("theta", "x", "b"):
        np.testing.assert_array_equal(res[0][key], res[1][key])
    assert res[0]["accepted"] == ref["accepted"]
    # the fp32 tile kernel's block partials group the samples differently on the shards (2e-6, as
    # the policy-gradient bound against the reference in test_gpu_update.py)
    assert cases.rel_l2(res[0]["b"], ref["b"]) <= 2e-6
    assert cases.rel_l2(res[0]["x"], ref["x"]) <= 1e-4
    assert cases.rel_l2(res[0]["theta"] - th, ref["theta"] - th) <= 1e-4
