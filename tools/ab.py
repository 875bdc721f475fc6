"""Interleaved A/B of library variants in ONE process (separate dlopen copies).
usage: python tools/ab.py lib1.so lib2.so[:ENV=V,ENV2=W] ...   (env SHAPES=arm,2x64 ROUNDS=5)
An optional ":ENV=V" suffix sets environment variables while that entry's contexts are created."""
import ctypes as C, os, sys, importlib, numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "trpo-robot-control_amd")]
specs = sys.argv[1:]
libs = [sp.split(":")[0] for sp in specs]
envs = [dict(kv.split("=") for kv in sp.split(":")[1].split(",")) if ":" in sp else {} for sp in specs]
mods = []
for i, path in enumerate(libs):
    os.environ["TRPO_LIB"] = path
    for m in [k for k in sys.modules if k.startswith("trpo_amd")]:
        del sys.modules[m]
    mod = importlib.import_module("trpo_amd")
    mod.lib()
    mods.append(mod)
from trpo_amd import synth
SH = {"arm": [15, 16, 16, 3], "2x64": [15, 64, 64, 3]}
for sname in os.environ.get("SHAPES", "arm,2x64").split(","):
    L = SH[sname]; n = int(os.environ.get("N", "50000"))
    th, obs = synth.make_theta(L), synth.make_obs(n, 15)
    P = synth.num_params(L); b = synth.make_b(P); v = synth.make_v(P)
    ctxs = []
    for m, env in zip(mods, envs):
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        c = m.Context(L, "lttl", th, obs, np.ones(3)); c.upload_b(b); c.upload_v(v); ctxs.append(c)
        for k, val in old.items():
            if val is None: os.environ.pop(k)
            else: os.environ[k] = val
    res = {i: {"cg": [], "k": [], "f": [], "k3": []} for i in range(len(mods))}
    xs = []
    for r in range(int(os.environ.get("ROUNDS", "5"))):
        for i, c in enumerate(ctxs):
            res[i]["cg"].append(c.time_ms(2, 20, 10, 0.0) * 1e3)
            c.upload_v(v)          # a CG rewrites the cooperative kernel's direction pack: the FVP rows below
                                   # time v as its upload packed it (the bench's C2 sequence)
            res[i]["k"].append(c.time_ms(0, 50) * 1e3)
            res[i]["f"].append(c.time_ms(1, 50) * 1e3)
            if sname == "arm":
                res[i]["k3"].append(c.time_ms(3, 10, 10) * 1e3)
    for i, c in enumerate(ctxs):
        x = c.cg(b, 10, 0.0); xs.append(x)
    for i, path in enumerate(libs):
        rel = np.linalg.norm(xs[i] - xs[0]) / np.linalg.norm(xs[0])
        print("%-5s %-40s cg10 med %.1f min %.1f us | fvp-kernel med %.2f us | fvp call med %.2f us | cg-iter kernel "
              "med %.2f us | x vs lib0 %.1e" % (
            sname, os.path.basename(specs[i]), np.median(res[i]["cg"]), np.min(res[i]["cg"]), np.median(res[i]["k"]),
            np.median(res[i]["f"]), np.median(res[i]["k3"]) if res[i]["k3"] else 0.0, rel), flush=True)
    for c in ctxs: c.close()
