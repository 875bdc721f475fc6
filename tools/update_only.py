"""Run N TRPO updates (armDOF_0 or 2x64, synthetic rollout) for kernel-trace profiling.
usage: python tools/update_only.py [arm|2x64] [n] [reps]"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "trpo-robot-control_amd")]
import trpo_amd
from trpo_amd import synth
shape = sys.argv[1] if len(sys.argv) > 1 else "arm"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 50000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
L = [15, 16, 16, 3] if shape == "arm" else [15, 64, 64, 3]
th = synth.make_theta(L)
obs = synth.make_obs(n, 15)
std = np.ones(3)
mean, action, adv = synth.make_rollout(L, "lttl", th, obs, std)
with trpo_amd.Context(L, "lttl", th, obs, std) as ctx:
    ctx.set_rollout(mean, action, adv)
    for _ in range(3):            # warm: first-call allocations, CG graph capture
        ctx.update()
    t0 = time.perf_counter()
    for _ in range(reps):
        r = ctx.update()
    print("%s n=%d update %.3f ms (accepted %d, cg_iters %d)" % (shape, n, 1e3 * (time.perf_counter() - t0) / reps,
                                                              r["accepted"], r["cg_iters"]))
