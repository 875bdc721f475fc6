"""The peer-window exchange (csrc/trpo_peer.hip) on ONE GPU: the one-shot all-reduce over xGMI that
replaces RCCL under the sharded CG (reference CG loop src/TRPO_CG.c:45-104 around the
per-sample FVP loop src/TRPO_FVP.c:771-921).

Two ways of running several ranks on one device:
  * in-process: contexts of one process, one thread per rank, windows joined by pointer
    (trpo_ctx_attach_peers_local) -- one exchange kernel per FVP, launched eagerly (contexts sharing
    a device must not allocate while another's exchange spins: see run_peer_ranks);
  * multi-process: one process per rank (tests/peer_worker.py), windows exported and opened as IPC
    handles (trpo_ctx_attach_peers) -- the path bench.py takes across GPUs, CG from its captured graph.
Checked: every rank ends with a bit-identical x (rank-order sums), x within the north-star bound of
the reference's golden and within rounding of the host-group exchange, standalone FVPs and the full
TRPO_Update through the generic in-place exchange, and that a rank that never arrives makes the
exchange give up with an error instead of hanging the GPU.
"""
import os
import subprocess
import sys
import tempfile
import threading

import numpy as np
import pytest

import cases
import oracle
import trpo_amd
from trpo_amd import synth

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
CG_TOL = 1e-4


def run_peer_ranks(ctxs, fn, timeout=120.0, warm=None):
    """Open every window, then attach and run fn(ctx, rank) on all contexts concurrently.
    warm(ctx): run once per context BEFORE attaching, so that the lazily sized device buffers exist
    already: in ONE process an allocation or free (which may wait for the whole device) in one
    rank's thread while another rank's exchange kernel spins for it would stall until the exchange's
    3 s timeout -- a hazard of contexts sharing one GPU, not of one process per GPU."""
    for c in ctxs:
        if warm is not None:
            warm(c)
        c.peer_handle()
    world = len(ctxs)
    out, err = [None] * world, [None] * world

    def work(r):
        try:
            ctxs[r].attach_peers_local(r, ctxs)
            out[r] = fn(ctxs[r], r)
        except BaseException as e:          # noqa: BLE001 -- reported below
            err[r] = e

    ts = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout)
    assert not any(t.is_alive() for t in ts), "a rank did not finish"
    for e in err:
        if e is not None:
            raise e
    return out


def _shards(x, bounds):
    return [trpo_amd.Context(x["layers"], x["acfunc"], x["theta"], x["obs"][lo:hi], x["std"], x["damping"])
            for lo, hi in bounds]


@pytest.mark.parametrize("bounds", [[(0, 25000), (25000, 50000)], [(0, 10000), (10000, 30001), (30001, 50000)]])
def test_peer_cg_lockstep_and_golden(bounds):
    c = cases.case("syn_arm_cg_n50000")
    x = cases.inputs(c)
    ctxs = _shards(x, bounds)
    try:
        res = run_peer_ranks(ctxs, lambda ctx, r: (ctx.cg(x["vin"], c["maxiter"], c["resth"]),
                                                   ctx.cg(x["vin"], c["maxiter"], c["resth"]),   # repeat
                                                   ctx.cg_history(), ctx.comm_info()),
                             warm=lambda ctx: ctx.cg(x["vin"], c["maxiter"], c["resth"]))
    finally:
        for ctx in ctxs:
            ctx.close()
    x0 = res[0][0]
    for r, (xa, xb, (rr, xn, it), info) in enumerate(res):
        np.testing.assert_array_equal(xa, x0)            # lockstep: identical bits on every rank
        np.testing.assert_array_equal(xb, x0)            # a second solve repeats the first
        assert it == c["iters"]
        assert info["rank"] == r and info["world"] == len(bounds)
        assert info["backend"].startswith("peer-xgmi"), info
    assert cases.rel_l2(x0, cases.expected(c)) <= CG_TOL


@pytest.mark.parametrize("proto", ["1", "3", "4"])
def test_peer_exchange_forms_agree(proto, monkeypatch):
    """The three forms of the exchange kernel (TRPO_PEER_PROTO, read when the window is created): 1 the
    flag hand-off with batched load rounds (the default through round 4), 3 the tagged granules on a
    compile-time world (the own rank's sum never travels), 4 the same with separate pushing and polling
    workgroups (the default since round 5).  Same rank-order sums => the CG solve (the replica-set
    exchange of the CG graph) and a standalone FVP (the in-place exchange) are bit-identical across the
    forms (checked against form 1 run here), on three ranks with ragged shards (slices that are not a
    multiple of the load round)."""
    c = cases.case("syn_arm_cg_n50000")
    x = cases.inputs(c)
    bounds = [(0, 10000), (10000, 30001), (30001, 50000)]

    def run(p):
        monkeypatch.setenv("TRPO_PEER_PROTO", p)
        ctxs = _shards(x, bounds)
        try:
            return run_peer_ranks(ctxs, lambda ctx, r: (ctx.cg(x["vin"], c["maxiter"], c["resth"]), ctx.fvp(x["vin"]),
                                                        ctx.comm_info()["backend"]),
                                  warm=lambda ctx: (ctx.cg(x["vin"], c["maxiter"], c["resth"]), ctx.fvp(x["vin"])))
        finally:
            for ctx in ctxs:
                ctx.close()

    ref = run("1")
    got = run(proto)
    for r in range(len(bounds)):
        np.testing.assert_array_equal(got[r][0], ref[0][0])     # CG: lockstep and equal to form 1
        np.testing.assert_array_equal(got[r][1], ref[0][1])     # standalone FVP (in-place exchange)
        assert ("tagged granules" in got[r][2]) == (proto in ("3", "4")), got[r][2]
    assert cases.rel_l2(got[0][0], cases.expected(c)) <= CG_TOL

    # a long message: the 2x64 policy's FVP (P = 5 443 > one load round of 4 x 256 elements; slices
    # of ~2 700 per rank > one round of 2 x 256) through the in-place exchange, vs one context
    L2, n = [15, 64, 64, 3], 6000
    th, obs, v = synth.make_theta(L2), synth.make_obs(n, L2[0]), synth.make_v(synth.num_params(L2))

    def run2(p):
        monkeypatch.setenv("TRPO_PEER_PROTO", p)
        ctxs = [trpo_amd.Context(L2, "lttl", th, obs[lo:hi], np.ones(3), 0.1) for lo, hi in ((0, 2500), (2500, n))]
        try:
            return run_peer_ranks(ctxs, lambda ctx, r: ctx.fvp(v), warm=lambda ctx: ctx.fvp(v))
        finally:
            for ctx in ctxs:
                ctx.close()

    z1, zp = run2("1"), run2(proto)
    with trpo_amd.Context(L2, "lttl", th, obs, np.ones(3), 0.1) as one:
        zone = one.fvp(v)
    for r in range(2):
        np.testing.assert_array_equal(zp[r], z1[0])
    assert cases.rel_l2(zp[0], zone) <= 1e-6


def test_peer_matches_host_group():
    """The same shards through the host-staged group: the exchange only changes the summation order
    (per-rank replica sums first), so the steps agree to rounding."""
    from test_gpu_shard import run_ranks
    c = cases.case("syn_arm_cg_n50000")
    x = cases.inputs(c)
    bounds = [(0, 20000), (20000, 50000)]
    ctxs = _shards(x, bounds)
    try:
        xg = run_ranks(ctxs, lambda ctx, r: ctx.cg(x["vin"], c["maxiter"], c["resth"]))[0]
    finally:
        for ctx in ctxs:
            ctx.close()
    ctxs = _shards(x, bounds)
    try:
        xp = run_peer_ranks(ctxs, lambda ctx, r: ctx.cg(x["vin"], c["maxiter"], c["resth"]),
                            warm=lambda ctx: ctx.cg(x["vin"], c["maxiter"], c["resth"]))[0]
    finally:
        for ctx in ctxs:
            ctx.close()
    assert cases.rel_l2(xp, xg) <= 1e-9


def test_peer_fvp_and_update():
    """Standalone FVP (atomic replica sets all-reduced in place) and TRPO_Update (policy-gradient,
    FVP(x) and surrogate sums) through the generic exchange, against one context over all samples."""
    c = cases.case("fix_fvp_n3150")
    x = cases.inputs(c)
    ctxs = _shards(x, [(0, 1000), (1000, 3150)])
    try:
        res = run_peer_ranks(ctxs, lambda ctx, r: ctx.fvp(x["vin"]), warm=lambda ctx: ctx.fvp(x["vin"]))
    finally:
        for ctx in ctxs:
            ctx.close()
    np.testing.assert_array_equal(res[0], res[1])
    assert cases.rel_l2(res[0], cases.expected(c)) <= 1e-5

    layers, n = [15, 16, 16, 3], 6000
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
        res = run_peer_ranks(ctxs, lambda ctx, r: ctx.update(), warm=lambda ctx: ctx.update())
    finally:
        for ctx in ctxs:
            ctx.close()
    for key in ("theta", "x", "b"):
        np.testing.assert_array_equal(res[0][key], res[1][key])
    assert res[0]["accepted"] == ref["accepted"]
    assert cases.rel_l2(res[0]["b"], ref["b"]) <= 2e-6
    assert cases.rel_l2(res[0]["x"], ref["x"]) <= 1e-4


@pytest.mark.parametrize("kind", ["2x64", "fp64"])
def test_peer_fvp_and_update_slab_paths(kind):
    """contexts WITHOUT atomic replica sets -- the 2x64 cooperative kernel (slab
    reduce) and the fp64 precision mode -- must all-reduce a standalone FVP and the update's FVP(x)
    under the peer exchange too; every rank then holds the global result (not its shard's), equal to
    one context over all samples."""
    layers = [15, 64, 64, 3] if kind == "2x64" else [15, 16, 16, 3]
    prec = "fp64" if kind == "fp64" else "fp32"
    n = 6000
    th, obs = synth.make_theta(layers), synth.make_obs(n, layers[0])
    std = np.ones(layers[-1])
    P = synth.num_params(layers)
    v = synth.make_v(P)
    mean, action, adv = synth.make_rollout(layers, "lttl", th, obs, std)
    with trpo_amd.Context(layers, "lttl", th, obs, std, 0.1, precision=prec) as one:
        zref = one.fvp(v)
        one.set_rollout(mean, action, adv)
        ref = one.update()
    bounds = [(0, 2500), (2500, n)]
    ctxs = [trpo_amd.Context(layers, "lttl", th, obs[lo:hi], std, 0.1, precision=prec) for lo, hi in bounds]
    for ctx, (lo, hi) in zip(ctxs, bounds):
        ctx.set_rollout(mean[lo:hi], action[lo:hi], adv[lo:hi])

    def work(ctx, r):
        return ctx.fvp(v), ctx.update()

    def warm(ctx):
        ctx.fvp(v)
        ctx.update()
    try:
        res = run_peer_ranks(ctxs, work, warm=warm)
    finally:
        for ctx in ctxs:
            ctx.close()
    np.testing.assert_array_equal(res[0][0], res[1][0])
    tol = 1e-12 if kind == "fp64" else 1e-5
    zor, _ = oracle.fvp(layers, "lttl", th, obs, std, v)
    e_one, e_peer, e_pair = cases.rel_l2(zref, zor), cases.rel_l2(res[0][0], zor), cases.rel_l2(res[0][0], zref)
    bad = np.nonzero(np.abs(res[0][0] - zor) > 1e-4 * np.abs(zor) + 1e-9)[0]
    assert e_one <= tol and e_peer <= tol and e_pair <= tol, (e_one, e_peer, e_pair, len(bad), bad[:40].tolist(),
                                                              bad[-10:].tolist(), (res[0][0][bad[:8]] / zor[bad[:8]]).tolist())
    for key in ("theta", "x", "b"):
        np.testing.assert_array_equal(res[0][1][key], res[1][1][key])
    assert res[0][1]["accepted"] == ref["accepted"]
    assert cases.rel_l2(res[0][1]["x"], ref["x"]) <= 1e-4


def test_peer_slab_paths_torch_runtime_first():
    """ADVICE r03 (high) / VERDICT r04 #2: in a process that imported torch FIRST (its bundled ROCm 7.0 HIP
    runtime then serves the library), contexts created after destroyed peer-attached contexts computed wrong
    FVPs until round 5; the trigger was returning the uncached peer window to that runtime, and the library
    now keeps such windows for the life of the process.  The round-4 reproduction -- the
    slab-path peer test twice, then a fresh single context -- must pass under that runtime."""
    env = dict(os.environ)
    env.pop("TRPO_PEER_FREE_WINDOW", None)
    r = subprocess.run([sys.executable, os.path.join(HERE, "peer_torch_first.py")], capture_output=True,
                       text=True, timeout=240, env=env)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert r.stdout.count("ok ") == 6, r.stdout


@pytest.mark.parametrize("proto", ["1", "4"])
def test_peer_missing_rank_times_out(proto, monkeypatch, capfd):
    """Only rank 0 of a world of 2 attaches: its exchange (the shard-size all-reduce of the attach)
    waits TRPO_PEER_WAIT_MS for rank 1, then gives up with an error -- the GPU is released, nothing hangs
    -- and says why on stderr: which rank, workgroup and exchange waited, for which
    peer's slot, and the tag it last read there (the flag form: the flag value)."""
    monkeypatch.setenv("TRPO_PEER_PROTO", proto)
    monkeypatch.setenv("TRPO_PEER_WAIT_MS", "500")
    c = cases.case("fix_fvp_n3150")
    x = cases.inputs(c)
    ctxs = _shards(x, [(0, 1000), (1000, 3150)])
    try:
        for ctx in ctxs:
            ctx.peer_handle()
        capfd.readouterr()
        with pytest.raises(trpo_amd.TRPOError):
            ctxs[0].attach_peers_local(0, ctxs)
        err = capfd.readouterr().err
    finally:
        for ctx in ctxs:
            ctx.close()
    assert "peer exchange timed out: rank 0 of 2" in err, err
    assert "exchange 1: after 0.5 s no data from rank 1" in err, err
    assert ("tag 0, expected 1; form %s" % proto) in err, err
    assert "rank 0 of 2 polls its window at" in err, err
    if proto == "4":
        # the pushing side (round 6): rank 0's pusher to rank 1 reports exchange 1 and where it went --
        # inside the window of rank 1 as attached in this process
        import re
        m = re.search(r"last pushed exchange 1 \((\d+) elements\) to rank 1 at (0x[0-9a-f]+) "
                      r"\(that window as attached here: (0x[0-9a-f]+)\)", err)
        assert m, err
        addr, base = int(m.group(2), 16), int(m.group(3), 16)
        assert base <= addr < base + (1 << 26), err


@pytest.mark.parametrize("world", [2, 4, 8])
def test_peer_ipc_processes(world):
    """One process per rank on the same GPU, windows exchanged as IPC handles through files: the
    8-rank case rehearses the protocol of an 8-GPU node (8 windows, 8 flag slots, rank-order sums)."""
    c = cases.case("syn_arm_cg_n50000")
    with tempfile.TemporaryDirectory() as tmp:
        procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "peer_worker.py"), str(r), str(world), tmp],
                                  stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
                 for r in range(world)]
        outs = []
        try:
            for p in procs:
                outs.append(p.communicate(timeout=150)[0])
        finally:
            for p in procs:
                if p.poll() is None:
                    p.kill()
        for p, o in zip(procs, outs):
            assert p.returncode == 0, o
        xs = [np.load(os.path.join(tmp, "x%d.npy" % r)) for r in range(world)]
        backends = [open(os.path.join(tmp, "backend%d.txt" % r)).read() for r in range(world)]
    for r in range(1, world):
        np.testing.assert_array_equal(xs[r], xs[0])
    assert all(b.startswith("peer-xgmi") for b in backends), backends
    assert cases.rel_l2(xs[0], cases.expected(c)) <= CG_TOL
