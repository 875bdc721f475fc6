"""Eager vs graph-replayed CG (TRPO_CG_GRAPH) inside the update path and for back-to-back solves,
armDOF_0 and 2x64 at N = 50k, interleaved in one process (the env is read at every CG enqueue)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "trpo-robot-control_amd")]
import numpy as np  # noqa: E402

import trpo_amd  # noqa: E402
from trpo_amd import synth  # noqa: E402

for L in ([15, 16, 16, 3], [15, 64, 64, 3]):
    n = 50000
    th, obs = synth.make_theta(L), synth.make_obs(n, L[0])
    std = np.ones(L[-1])
    mean, action, adv = synth.make_rollout(L, "lttl", th, obs, std)
    b = synth.make_b(synth.num_params(L))
    res = {}
    with trpo_amd.Context(L, "lttl", th, obs, std, 0.1) as ctx:
        ctx.set_rollout(mean, action, adv)
        ctx.upload_b(b)
        for rnd in range(4):
            for form in ("eager", "graph"):
                os.environ["TRPO_CG_GRAPH"] = "1" if form == "graph" else "0"
                for _ in range(3):
                    ctx.update()
                t0 = time.perf_counter()
                for _ in range(20):
                    ctx.update()
                tu = (time.perf_counter() - t0) / 20
                ctx.upload_b(b)
                tc = ctx.time_ms(2, 50, 10, 0.0)
                res.setdefault(form, []).append((1e3 * tu, tc))
    for form, v in res.items():
        print("%s %-5s update med %.3f ms | back-to-back CG10 med %.4f ms" % (L, form, np.median([a for a, _ in v]),
                                                                           np.median([c for _, c in v])), flush=True)
