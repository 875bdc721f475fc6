"""Diagnostic: two shard contexts of one process on one GPU (host group or peer windows), 2x64 slab
path, the full update and its stages repeated -- do the ranks stay bit-identical?  Prints, per trial,
which stage first differs (policy gradient b, CG x, FVP z, update theta)."""
import os, sys
R = os.path.join(os.path.dirname(__file__), "..", "..")
sys.path[:0] = [os.path.join(R, "tests"), os.path.join(R, "trpo-robot-control_amd"), os.path.join(R, "oracle")]
import numpy as np
import trpo_amd
from trpo_amd import synth
from test_gpu_shard import run_ranks
from test_gpu_peer import run_peer_ranks
mode = sys.argv[1] if len(sys.argv) > 1 else "group"
trials = int(sys.argv[2]) if len(sys.argv) > 2 else 8
L = [15, 64, 64, 3]
n = 6000
th, obs = synth.make_theta(L), synth.make_obs(n, L[0])
std = np.ones(3)
P = synth.num_params(L)
v, b = synth.make_v(P), synth.make_b(P)
mean, action, adv = synth.make_rollout(L, "lttl", th, obs, std)
bounds = [(0, 2500), (2500, n)]
bad = 0
for trial in range(trials):
    ctxs = [trpo_amd.Context(L, "lttl", th, obs[lo:hi], std, 0.1) for lo, hi in bounds]
    for ctx, (lo, hi) in zip(ctxs, bounds):
        ctx.set_rollout(mean[lo:hi], action[lo:hi], adv[lo:hi])

    def work(c, r):
        out = {}
        out["pg"] = c.policy_gradient()[0] if hasattr(c, "policy_gradient") else None
        out["cg"] = c.cg(b, 10, 0.0)
        out["fvp"] = c.fvp(v)
        u = c.update()
        out.update(ub=u["b"], ux=u["x"], uth=u["theta"])
        out["cg2"] = c.cg(b, 10, 0.0)
        return out
    try:
        if mode == "group":
            res = run_ranks(ctxs, work)
        else:
            res = run_peer_ranks(ctxs, work, warm=lambda c: (c.fvp(v), c.update()))
    finally:
        for c in ctxs:
            c.close()
    diff = [k for k in ("pg", "cg", "fvp", "ub", "ux", "uth", "cg2") if res[0][k] is not None
            and not np.array_equal(res[0][k], res[1][k])]
    if diff:
        bad += 1
        k = diff[0]
        d = np.nonzero(res[0][k] != res[1][k])[0]
        print("trial", trial, "DIFF in", diff, "first", k, "n", len(d), "idx", d[:10].tolist(),
              "max rel", float(np.max(np.abs(res[0][k] - res[1][k]) / (np.abs(res[1][k]) + 1e-30))), flush=True)
    else:
        print("trial", trial, "equal", flush=True)
print("bad", bad, "of", trials)
