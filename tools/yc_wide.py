"""Debug: forward cache on the 1x4x4x1 one-wave-per-tile kernel (TRPO_COOP=0)."""
import os, sys, numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, "trpo-robot-control_amd"), os.path.join(R, "tests"), os.path.join(R, "oracle")]
os.environ["TRPO_COOP"] = "0"
import trpo_amd, cases
c = cases.case("syn_2x64_fvp_n4096"); x = cases.inputs(c); e = cases.expected(c)
os.environ["TRPO_YCACHE"] = "0"
with trpo_amd.Context(x["layers"], x["acfunc"], x["theta"], x["obs"], x["std"], x["damping"]) as ctx:
    z0 = ctx.fvp(x["vin"])
os.environ["TRPO_YCACHE"] = "1"
for n in (4096, 2048, 1024):
  for blocks in ("0", "8", "64"):
    os.environ["TRPO_FVP_BLOCKS"] = blocks
    with trpo_amd.Context(x["layers"], x["acfunc"], x["theta"], x["obs"][:n], x["std"], x["damping"]) as ctx:
        r = ctx.fvp(x["vin"])
        z = [ctx.fvp(x["vin"]) for _ in range(5)]
        print(n, blocks, ctx.geometry, ["%.1e" % cases.rel_l2(q, r) for q in z], flush=True)
