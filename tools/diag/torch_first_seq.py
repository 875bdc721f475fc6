"""Replays tests/test_gpu_peer.py::test_peer_fvp_and_update_slab_paths's single-context steps exactly,
torch imported first, and breaks a wrong FVP down by parameter block.  usage: ... [torch|notorch] [reps]"""
import os
import sys

if len(sys.argv) > 1 and sys.argv[1] == "torch":
    import torch  # noqa: F401
R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path[:0] = [os.path.join(R, "tests"), os.path.join(R, "trpo-robot-control_amd"), os.path.join(R, "oracle")]
import warnings  # noqa: E402

warnings.simplefilter("ignore", RuntimeWarning)
import numpy as np  # noqa: E402

import trpo_amd  # noqa: E402

trpo_amd.lib()
import oracle  # noqa: E402
from trpo_amd import synth  # noqa: E402

print("runtime", trpo_amd.runtime_path(), flush=True)
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3


def blocks(L):
    out, pos = [], 0
    for i in range(len(L) - 1):
        out.append(("W%d" % i, pos, pos + L[i] * L[i + 1]))
        pos += L[i] * L[i + 1]
        out.append(("b%d" % i, pos, pos + L[i + 1]))
        pos += L[i + 1]
    out.append(("logstd", pos, pos + L[-1]))
    return out


for rep in range(reps):
    for kind in ("2x64", "fp64"):
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
            zdev = one.download_z()
            zref2 = one.fvp(v)
            one.set_rollout(mean, action, adv)
            one.update()
            zref3 = one.fvp(v)
        zor, _ = oracle.fvp(layers, "lttl", th, obs, std, v)
        e = lambda a: float(np.linalg.norm(a - zor) / np.linalg.norm(zor))  # noqa: E731
        line = "rep %d %s: fvp#1 %.2e (dev %.2e) fvp#2 %.2e after-update %.2e" % (rep, kind, e(zref), e(zdev), e(zref2),
                                                                              e(zref3))
        if e(zref) > 1e-5:
            d = zref - zor
            line += " | by block: " + " ".join("%s %.1e" % (nm, np.linalg.norm(d[a:b]) / max(np.linalg.norm(zor[a:b]), 1e-300))
                                               for nm, a, b in blocks(layers))
            lam = (zref - zor) / np.where(np.abs(v) > 0, v, 1)
            line += " | (z-zor)/v median %.4g" % float(np.median(lam))
        print(line, flush=True)
