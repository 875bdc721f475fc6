import os, sys, numpy as np
sys.path[:0] = ["tests", "trpo-robot-control_amd", "oracle"]
import cases, trpo_amd
def run(name, note=""):
    c = cases.case(name); x = cases.inputs(c)
    with trpo_amd.Context(x["layers"], x["acfunc"], x["theta"], x["obs"], x["std"], x["damping"]) as ctx:
        out = ctx.fvp(x["vin"]) if c["kind"] == "fvp" else ctx.cg(x["vin"], c["maxiter"], c["resth"])
        out2 = ctx.fvp(x["vin"]) if c["kind"] == "fvp" else out
        print(note, name, ctx.kernel_name, ctx.geometry, "rel=%.3e rel2=%.3e" % (cases.rel_l2(out, cases.expected(c)), cases.rel_l2(out2, cases.expected(c))), flush=True)
seq = sys.argv[1].split(",")
for s in seq: run(s)
