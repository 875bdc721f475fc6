"""Distributed vs fused cooperative CG step: per-iteration rdotr history and the final x against the
oracle, for a few shapes / precisions (TRPO_COOP_DIST=1 / 0)."""
import os, sys
sys.path[:0] = ['oracle', 'trpo-robot-control_amd']
import numpy as np
import oracle, trpo_amd
from trpo_amd import synth
cases = [([32, 16, 16, 1], "lotl", "fp64"), ([32, 16, 16, 1], "lotl", "fp32"), ([32, 16, 16, 1], "lttl", "fp64"),
         ([15, 16, 16, 1], "lotl", "fp64"), ([32, 16, 16, 3], "lttl", "fp64"), ([30, 64, 64, 4], "ltts", "fp64")]
for layers, acts, prec in cases:
    n = 2345
    th, obs = synth.make_theta(layers), synth.make_obs(n, layers[0])
    std = np.linspace(0.8, 1.1, layers[-1])
    P = synth.num_params(layers)
    b = synth.make_b(P)
    ref = oracle.cg(layers, acts, th, obs, std, b, 10, 0.0)
    row = []
    for dist in ("1", "0"):
        os.environ["TRPO_COOP_DIST"] = dist
        with trpo_amd.Context(layers, acts, th, obs, std, precision=prec) as ctx:
            x = ctx.cg(b, 10, 0.0)
            rr, xn, it = ctx.cg_history()
            row.append((np.linalg.norm(x - ref["x"]) / np.linalg.norm(ref["x"]), rr[:4], ctx.kernel_name))
    print(layers, acts, prec, "dist relL2 %.2e fused %.2e" % (row[0][0], row[1][0]), row[0][2])
    print("   rr dist ", row[0][1]); print("   rr fused", row[1][1]); print("   rr ref  ", ref["rdotr"][:4] if "rdotr" in ref else "")
