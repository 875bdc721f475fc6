"""the forward-cache (MODE 2/3) variant of the 1x4x4x1 one-wave-per-tile kernel
spills to scratch; round 1 saw its runs differ bit-wise.  Loads the diagnostic build
(make variant NAME=yc1441 DEFS="-DTRPO_DIAG_1441 -DTRPO_YC_ALL=1") and checks repeatability: the
same FVP / CG several times in one process, cached vs recomputing (TRPO_YCACHE=0), and against the
oracle; on a mismatch prints the first differing parameters and their pack / accumulator slots."""
import os, sys
R = os.path.join(os.path.dirname(__file__), "..", "..")
os.environ["TRPO_LIB"] = os.path.join(R, "trpo-robot-control_amd", "lib", "variants", "yc1441.so")
os.environ["TRPO_COOP"] = "0"
sys.path[:0] = [os.path.join(R, "tests"), os.path.join(R, "trpo-robot-control_amd"), os.path.join(R, "oracle")]
import numpy as np
import cases, oracle, trpo_amd
from trpo_amd import synth
L = [15, 64, 64, 3]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
th, obs = synth.make_theta(L), synth.make_obs(n, 15)
std = np.ones(3)
P = synth.num_params(L)
v, b = synth.make_v(P), synth.make_b(P)
zr, _ = oracle.fvp(L, "lttl", th, obs, std, v)
res = {}
for yc in ("1", "0"):
    os.environ["TRPO_YCACHE"] = yc
    with trpo_amd.Context(L, "lttl", th, obs, std, 0.1) as c:
        print("kernel", c.kernel_name, "ycache", yc, flush=True)
        zs = [c.fvp(v) for _ in range(6)]
        xs = [c.cg(b, 10, 0.0) for _ in range(4)]
    res[yc] = (zs, xs)
    for i, z in enumerate(zs):
        d = np.nonzero(z != zs[0])[0]
        print(" fvp", i, "relL2 vs oracle %.2e" % cases.rel_l2(z, zr), "differs from fvp0 at", len(d), d[:12].tolist(), flush=True)
    for i, x in enumerate(xs):
        d = np.nonzero(x != xs[0])[0]
        print(" cg", i, "differs from cg0 at", len(d), d[:12].tolist(), flush=True)
for i in range(6):
    d = np.nonzero(res["1"][0][i] != res["0"][0][0])[0]
    print("cached fvp", i, "vs recompute fvp0: differ at", len(d), d[:12].tolist())
