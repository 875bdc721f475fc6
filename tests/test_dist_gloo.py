"""world_size-2 gloo check of the sharded FVP/CG decomposition the RCCL path uses:
per-rank partial sums over contiguous shards, one sum all-reduce per FVP, division by the
global N, replicated fp64 CG -- must equal the single-process reference CG."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import cases


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


def test_shard_range_covers_exactly():
    from trpo_amd.dist import shard_range
    for n in (0, 1, 7, 50000):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1
