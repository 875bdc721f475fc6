"""GPU diagnostic: the fp32 device CG's rdotr history next to the reference's fp64 one
(the oracle, pinned to src/TRPO_CG.c) for every CG / update golden and every random draw, with the step
error -- to find a statistic of the device's own trajectory that marks the solves whose fp32 step is
not the reference's.  Prints one block per case."""
import os
import sys

R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path[:0] = [os.path.join(R, "tests"), os.path.join(R, "trpo-robot-control_amd"), os.path.join(R, "oracle")]
import numpy as np  # noqa: E402

import trpo_amd  # noqa: E402

trpo_amd.lib()
import cases  # noqa: E402
import oracle  # noqa: E402
from trpo_amd import synth  # noqa: E402
from test_gpu_random_shapes import _draw  # noqa: E402


def one(name, layers, acts, th, obs, std, b, maxiter, resth, damping=0.1):
    ref = oracle.cg(layers, acts, th, obs, std, b, maxiter, resth, damping, verbose=False)
    with trpo_amd.Context(layers, acts, th, obs, std, damping) as c:
        os.environ["TRPO_RITZ_RERUN"] = "0"            # the fp32 solve as it is (no fp64 re-solve)
        x = c.cg(b, maxiter, resth)
        st = c.cg_status()
        os.environ.pop("TRPO_RITZ_RERUN")
        rr, xn, it = c.cg_history()
    e = np.linalg.norm(x - ref["x"]) / np.linalg.norm(ref["x"])
    h = ref.get("rdotr")
    print("%s  err %.2e  iters dev %d ref %s  orth_loss %.3e  ritz %.3e" % (name, e, it, ref.get("iters"),
                                                                         st["orth_loss"], st["ritz_residual"]))
    print("   dev rdotr  " + " ".join("%.2e" % v for v in rr))
    if h is not None:
        print("   ref rdotr  " + " ".join("%.2e" % v for v in h))
    print("   dev ratios " + " ".join("%.3f" % (rr[i + 1] / rr[i]) for i in range(len(rr) - 1)), flush=True)


for name in ("fix_cg_n3150_th1e-10", "fix_cg_n3150_th0", "fix_cg_n2400_th1e-10", "syn_sigma_cg", "syn_arm_cg_n50000",
             "syn_2x64_cg_n50000"):
    c = cases.case(name)
    X = cases.inputs(c)
    one(name, X["layers"], X["acfunc"], X["theta"], X["obs"], X["std"], X["vin"], c["maxiter"], c["resth"],
        X["damping"])
for name in ("fix_update_n3150", "syn_update_sigma_n5000", "syn_update_arm_n20000", "syn_update_2x64_n8192"):
    c = cases.case(name)
    X = cases.update_inputs(c)
    b, _ = oracle.policy_grad(X["layers"], X["acfunc"], X["theta"], X["obs"], X["mean"], X["action"], X["adv"])
    one(name, X["layers"], X["acfunc"], X["theta"], X["obs"], X["std"], b, 10, 1e-10, X["damping"])
for seed in range(36):
    layers, acts, n, std = _draw(seed)
    th = synth.make_theta(layers, seed=100 + seed)
    obs = synth.make_obs(n, layers[0], seed=200 + seed)
    mean, action, adv = synth.make_rollout(layers, acts, th, obs, std, seed=500 + seed)
    b, _ = oracle.policy_grad(layers, acts, th, obs, mean, action, adv)
    one("draw %d %s %s" % (seed, layers, acts), layers, acts, th, obs, std, b, 10, 1e-10)
