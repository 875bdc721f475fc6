"""tests/peer_torch_first.py fails deterministically in its SECOND repetition: the single-context 2x64 FVP
is 1.98e-3 off after the first repetition's in-process peer ranks ran.  Which step of those leaves the
state behind?  usage: ... [torch|notorch] STAGE   (STAGE: none | create | handle | attach | fvp | update | threads |
group | seqpeer)
  threads: the two contexts NOT attached, fvp + update concurrently from two threads
  group:   attached to an in-process host group instead of peer windows, fvp + update concurrently
optional 3rd argument "keep": the two contexts stay open while the later single context runs (round 5:
does the later context go wrong only when it can reuse their freed memory?)"""
import os
import sys

if sys.argv[1] == "torch":
    import torch  # noqa: F401
R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path[:0] = [os.path.join(R, "tests"), os.path.join(R, "trpo-robot-control_amd"), os.path.join(R, "oracle")]
import warnings  # noqa: E402

warnings.simplefilter("ignore", RuntimeWarning)
import numpy as np  # noqa: E402

import trpo_amd  # noqa: E402

trpo_amd.lib()
import oracle  # noqa: E402
from test_gpu_peer import run_peer_ranks  # noqa: E402
from trpo_amd import synth  # noqa: E402

stage = sys.argv[2]
layers = [15, 64, 64, 3]
n = 6000
th, obs = synth.make_theta(layers), synth.make_obs(n, layers[0])
std = np.ones(3)
v = synth.make_v(synth.num_params(layers))
mean, action, adv = synth.make_rollout(layers, "lttl", th, obs, std)
zor, _ = oracle.fvp(layers, "lttl", th, obs, std, v)


def single(tag):
    with trpo_amd.Context(layers, "lttl", th, obs, std, 0.1) as one:
        z = one.fvp(v)
        zd = one.download_z()
        z2 = one.fvp(v)
    print("%s: fvp %.2e dev %.2e again %.2e" % (tag, np.linalg.norm(z - zor) / np.linalg.norm(zor),
                                                np.linalg.norm(zd - zor) / np.linalg.norm(zor),
                                                np.linalg.norm(z2 - zor) / np.linalg.norm(zor)), flush=True)


single("before")
if stage != "none":
    bounds = [(0, 2500), (2500, n)]
    ctxs = [trpo_amd.Context(layers, "lttl", th, obs[lo:hi], std, 0.1) for lo, hi in bounds]
    for c, (lo, hi) in zip(ctxs, bounds):
        c.set_rollout(mean[lo:hi], action[lo:hi], adv[lo:hi])
    if stage in ("handle", "attach", "fvp", "update"):
        for c in ctxs:
            c.fvp(v)
            c.update()
            c.peer_handle()
    if stage in ("attach", "fvp", "update"):
        work = {"attach": lambda c, r: None, "fvp": lambda c, r: c.fvp(v),
                "update": lambda c, r: (c.fvp(v), c.update())}[stage]
        run_peer_ranks_nowarm = run_peer_ranks
        import threading
        out = [None, None]

        def go(r):
            ctxs[r].attach_peers_local(r, ctxs)
            out[r] = work(ctxs[r], r)
        ts = [threading.Thread(target=go, args=(r,)) for r in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    if stage in ("threads", "group"):
        import threading
        g = trpo_amd.Group(2) if stage == "group" else None

        def go2(r):
            if g is not None:
                ctxs[r].attach_group(g, r)
            ctxs[r].fvp(v)
            ctxs[r].update()
        ts = [threading.Thread(target=go2, args=(r,)) for r in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    keep = len(sys.argv) > 3 and sys.argv[3] == "keep"
    if not keep:
        for c in ctxs:
            c.close()
single("after %s" % stage)
single("after %s, again" % stage)
if stage != "none" and keep:
    for c in ctxs:
        c.close()
    single("after %s, contexts closed" % stage)
