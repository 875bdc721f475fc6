"""The RCCL code path on one GPU: a context attached to a one-rank communicator runs every
collective the sharded path issues (the FVP partial all-reduce, captured into the CG graph; the
policy-gradient and surrogate all-reduces of the update), and must give the results of the
communicator-free context.  World size 1 makes the sums identities, so the comparison is exact
up to the launch-sequence differences (the communicator-free FVP call fuses its epilogue into
the slab reduce; with a communicator the epilogue runs after the all-reduce).  The multi-rank
decomposition itself is checked on CPU (tests/test_dist_gloo.py); 2/4/8-GPU runs are the
driver's."""
import numpy as np
import pytest

import cases
import trpo_amd
from trpo_amd import synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("layers,precision", [([15, 16, 16, 3], "fp32"), ([15, 64, 64, 3], "fp32"),
                                              ([15, 64, 64, 3], "fp64"), ([15, 16, 16, 16, 3], "fp32")])
def test_one_rank_communicator_matches_plain_context(layers, precision):
    from trpo_amd import synth
    if precision == "fp64" and len(layers) != 4:
        pytest.skip("fp64 needs a tile kernel")
    acts = "l" + "t" * (len(layers) - 2) + "l"
    n = 3000
    th, obs = synth.make_theta(layers), synth.make_obs(n, layers[0])
    std = np.linspace(0.8, 1.1, layers[-1])
    P = synth.num_params(layers)
    v, b = synth.make_v(P), synth.make_b(P)
    mean, action, adv = synth.make_rollout(layers, acts, th, obs, std)
    res = []
    for attach in (False, True):
        with trpo_amd.Context(layers, acts, th, obs, std, precision=precision) as ctx:
            if attach:
                ctx.attach_comm(0, 1, trpo_amd.unique_id())
            f = ctx.fvp(v)
            x = ctx.cg(b, 10, 0.0)
            x2 = ctx.cg(b, 10, 0.0)                  # graph replay (captured with the collective)
            ctx.set_rollout(mean, action, adv)
            r = ctx.update()
            res.append((f, x, x2, r))
    (f0, x0, x20, r0), (f1, x1, x21, r1) = res
    assert cases.rel_l2(f1, f0) <= 1e-14
    np.testing.assert_array_equal(x1, x21)
    np.testing.assert_array_equal(x0, x20)
    assert cases.rel_l2(x1, x0) <= 1e-12
    assert cases.rel_l2(r1["theta"], r0["theta"]) <= 1e-12
    assert r1["accepted"] == r0["accepted"]


@pytest.mark.parametrize("used", ["1", "2", "5"])
def test_fewer_replicas_same_result(used, monkeypatch):
    """Under RCCL the CG uses fewer atomic replicas (sized from the largest shard) so the per-FVP
    all-reduce stays small.  fp32 block partials are added into fp64 exactly, so the replica count
    must not change the result: forced on one GPU, FVP and CG agree bit for bit."""
    L = [15, 16, 16, 3]
    P = synth.num_params(L)
    th, obs = synth.make_theta(L), synth.make_obs(20000, 15)
    v, b = synth.make_v(P), synth.make_b(P)
    out = []
    for env in (None, used):
        if env:
            monkeypatch.setenv("TRPO_REPLICAS_USED", env)
        with trpo_amd.Context(L, "lttl", th, obs, np.ones(3), 0.1) as ctx:
            out.append((ctx.fvp(v), ctx.fvp(v), ctx.cg(b, 10, 0.0)))
    for a, c in zip(out[0], out[1]):
        np.testing.assert_array_equal(a, c)
