"""world_size-2 gloo check of the sharded FVP/CG decomposition the RCCL path uses:
per-rank partial sums over contiguous shards, one sum all-reduce per FVP, division by the
global N, replicated fp64 CG -- must equal the single-process reference CG."""
import os
import socket

import numpy as np
import pytest

import cases

# torch is imported inside the functions only: a module-level import would load torch's bundled
# libamdhip64.so.7 into every pytest process that merely COLLECTS this file, including the GPU runs
# (-m gpu), where libtrpo_mi355x.so must run on the system ROCm runtime (trpo_amd.lib()).


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "trpo-robot-control_amd"), os.path.join(root, "oracle"),
                    os.path.join(root, "tests")]
    import torch
    import torch.distributed as dist
    import oracle
    from trpo_amd import synth
    from trpo_amd.dist import shard_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    L, n, lam = [15, 16, 16, 3], 3000, 0.1
    th, obs = synth.make_theta(L), synth.make_obs(n, 15)
    std = np.array([0.6065306597126334, 0.8, 1.3])
    P = synth.num_params(L)
    nw = P - L[-1]
    lo, hi = shard_range(n, rank, world)

    def fvp(v):
        out, _ = oracle.fvp(L, "lttl", th, obs[lo:hi], std, v, damping=0.0)
        part = torch.tensor(out[:nw] * (hi - lo))          # un-normalised local sum
        dist.all_reduce(part)                              # the one exchange per FVP
        z = np.empty(P)
        z[:nw] = part.numpy() / n + lam * v[:nw]
        z[nw:] = 2 * v[nw:] + lam * v[nw:]
        return z

    b = synth.make_b(P)
    x, r, p = np.zeros(P), b.copy(), b.copy()
    rr = r @ r
    for _ in range(10):                                    # src/TRPO_CG.c:45-104, replicated
        z = fvp(p)
        a = rr / (p @ z)
        x += a * p
        r -= a * z
        nr = r @ r
        p = r + (nr / rr) * p
        rr = nr
    xs = [torch.zeros(P, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(xs, torch.tensor(x))
    if rank == 0:
        ref = oracle.cg(L, "lttl", th, obs, std, b, 10, 0.0, lam)["x"]
        q.put((cases.rel_l2(x, ref), max(float(np.abs(xs[0].numpy() - xi.numpy()).max()) for xi in xs)))
    dist.destroy_process_group()


def test_sharded_cg_two_ranks_gloo():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    rel, spread = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert rel < 1e-7           # same algorithm, fp64; only the shard summation order differs (CG amplifies it)
    assert spread == 0.0        # replicated CG stays bit-identical on every rank


def _update_worker(rank, world, port, q):
    """Sharded TRPO_Update as the RCCL path runs it: per-rank policy-gradient, FVP and
    surrogate partial sums over the rank's shard, one sum all-reduce each, then the
    replicated fp64 CG / step size / line search on every rank."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "trpo-robot-control_amd"), os.path.join(root, "oracle"),
                    os.path.join(root, "tests")]
    import torch
    import torch.distributed as dist
    import oracle
    from trpo_amd import synth
    from trpo_amd.dist import shard_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    L, n, lam = [15, 16, 16, 3], 3000, 0.1
    th = synth.make_theta(L)
    th[-3:] = [-0.5, 0.0, 0.25]
    std = np.array([0.6065306597126334, 1.0, 1.2840254166877414])
    obs = synth.make_obs(n, 15)
    mean, action, adv = synth.make_rollout(L, "lttl", th, obs, std)
    P, nw = synth.num_params(L), synth.num_params(L) - 3
    lo, hi = shard_range(n, rank, world)
    sh = lambda a: a[lo:hi]

    def allsum(a):
        t = torch.tensor(np.atleast_1d(np.asarray(a, dtype=np.float64)))
        dist.all_reduce(t)
        return t.numpy()

    # policy gradient + sum(adv): one all-reduce of P + 1 values (src/TRPO_Update.c:254-378)
    bs, asum = oracle.policy_grad(L, "lttl", th, sh(obs), sh(mean), sh(action), sh(adv), normalise=False)
    red = allsum(np.concatenate([bs, [asum]]))
    b, fval = red[:P] / n, -red[P] / n

    def fvp(v):
        out, _ = oracle.fvp(L, "lttl", th, sh(obs), std, v, damping=0.0)
        part = allsum(out[:nw] * (hi - lo))
        z = np.empty(P)
        z[:nw] = part / n + lam * v[:nw]
        z[nw:] = 2 * v[nw:] + lam * v[nw:]
        return z

    x, r, p = np.zeros(P), b.copy(), b.copy()
    rr = r @ r
    for _ in range(10):
        if rr < 1e-10:
            break
        z = fvp(p)
        a = rr / (p @ z)
        x += a * p
        r -= a * z
        nr = r @ r
        p = r + (nr / rr) * p
        rr = nr
    shs = 0.5 * (fvp(x) @ x)
    lm = np.sqrt(shs / 0.01)
    full = x / lm
    rate = (b @ x) / lm
    theta = x.copy()
    for k in range(10):
        frac = 0.5 ** k
        cand = th + frac * full
        s = allsum(oracle.surrogate_sum(L, "lttl", cand, sh(obs), sh(mean), sh(action), sh(adv), std))[0]
        actual = fval + s / n
        if actual / (rate * frac) > 0.1 and actual > 0:
            theta = cand
            break
    if rank == 0:
        ref = oracle.update(L, "lttl", th, obs, mean, action, adv, std, lam)
        q.put(cases.rel_l2(theta - th, ref["theta"] - th))
    dist.destroy_process_group()


def test_sharded_update_two_ranks_gloo():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_update_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    rel = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert rel < 1e-7


def test_shard_range_covers_exactly():
    from trpo_amd.dist import shard_range
    for n in (0, 1, 7, 50000):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1
