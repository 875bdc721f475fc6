import sys, numpy as np
sys.path[:0] = ["tests", "trpo-robot-control_amd", "oracle"]
import cases, trpo_amd
for name in ["fix_cg_n3150_th1e-10", "fix_cg_n3150_th0", "syn_arm_cg_n50000", "syn_2x64_cg_n50000"]:
    c = cases.case(name); x = cases.inputs(c)
    with trpo_amd.Context(x["layers"], x["acfunc"], x["theta"], x["obs"], x["std"], x["damping"]) as ctx:
        out = ctx.cg(x["vin"], c["maxiter"], c["resth"])
        rr, xn, it = ctx.cg_history()
        print(name, ctx.kernel_name, ctx.geometry, "relL2", cases.rel_l2(out, cases.expected(c)), "iters", it, c["iters"])
        for i in range(len(rr)):
            ref = c["rdotr"][i] if i < len(c["rdotr"]) else float("nan")
            print("  %2d  %.6e  %.6e   xn %.10e %.10e" % (i, rr[i], ref, xn[i], c["xnorm"][i] if i < len(c["xnorm"]) else np.nan))
