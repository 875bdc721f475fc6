"""Device CG step vs the reference goldens, residual reorthogonalisation on and off (TRPO_CG_REORTH),
fp32 and fp64: the table of DESIGN §3.  GPU; prints one line per case."""
import os
import sys

sys.path[:0] = ['tests', 'oracle', 'trpo-robot-control_amd']
import cases  # noqa: E402
import trpo_amd  # noqa: E402


def run(c, reorth, prec):
    os.environ["TRPO_CG_REORTH"] = reorth
    if c["kind"] == "update":
        x = cases.update_inputs(c)
        with trpo_amd.Context(x["layers"], x["acfunc"], x["theta"], x["obs"], x["std"], x["damping"],
                              precision=prec) as ctx:
            ctx.set_rollout(x["mean"], x["action"], x["adv"])
            r = ctx.update()
            exp = cases.expected(c)
            th = x["theta"]
            d = cases.rel_l2(r["theta"] - th, exp - th) if c["accepted"] >= 0 else cases.rel_l2(r["theta"], exp)
            return d, r["cg_iters"]
    x = cases.inputs(c)
    with trpo_amd.Context(x["layers"], x["acfunc"], x["theta"], x["obs"], x["std"], x["damping"],
                          precision=prec) as ctx:
        out = ctx.cg(x["vin"], c["maxiter"], c["resth"])
        return cases.rel_l2(out, cases.expected(c)), ctx.cg_history()[2]


for c in cases.manifest():
    if c["kind"] not in ("cg", "update"):
        continue
    row = [c["name"], "ref_iters=%d" % c["iters"]]
    for prec in ("fp32", "fp64"):
        if prec == "fp64" and len(c.get("layers", [15, 16, 16, 3])) != 4:
            continue
        for ro in ("1", "0"):
            d, it = run(c, ro, prec)
            row.append("%s reorth=%s %.3e (%d it)" % (prec, ro, d, it))
    print(" | ".join(row), flush=True)
