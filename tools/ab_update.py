"""Interleaved A/B of whole TRPO updates across library builds (separate dlopen copies, one
process): median wall time per update and bitwise comparison of theta / x / line-search values.
usage: python tools/ab_update.py lib1.so lib2.so ...   (env SHAPES=arm,2x64 N=50000 ROUNDS=5)"""
import importlib, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "trpo-robot-control_amd")]
libs = sys.argv[1:]
mods = []
for path in libs:
    os.environ["TRPO_LIB"] = path
    for m in [k for k in sys.modules if k.startswith("trpo_amd")]:
        del sys.modules[m]
    mod = importlib.import_module("trpo_amd")
    mod.lib()
    mods.append(mod)
from trpo_amd import synth
SH = {"arm": [15, 16, 16, 3], "2x64": [15, 64, 64, 3]}
n = int(os.environ.get("N", "50000"))
for sname in os.environ.get("SHAPES", "arm,2x64").split(","):
    L = SH[sname]
    th, obs, std = synth.make_theta(L), synth.make_obs(n, L[0]), np.ones(L[-1])
    mean, action, adv = synth.make_rollout(L, "lttl", th, obs, std)
    ctxs = []
    for m in mods:
        c = m.Context(L, "lttl", th, obs, std)
        c.set_rollout(mean, action, adv)
        for _ in range(3):
            c.update()
        ctxs.append(c)
    times = [[] for _ in mods]
    for _ in range(int(os.environ.get("ROUNDS", "5"))):
        for i, c in enumerate(ctxs):
            t0 = time.perf_counter()
            for _ in range(5):
                c.update()
            times[i].append((time.perf_counter() - t0) / 5 * 1e3)
    outs = [c.update() for c in ctxs]
    for i, path in enumerate(libs):
        same = all(np.array_equal(outs[i][k], outs[0][k]) for k in ("theta", "x", "actual", "expected"))
        print("%-5s %-30s update med %.3f ms min %.3f ms | evaluated %d | bitwise == lib0: %s" % (
            sname, os.path.basename(path), np.median(times[i]), np.min(times[i]), outs[i]["evaluated"], same),
            flush=True)
    for c in ctxs:
        c.close()
