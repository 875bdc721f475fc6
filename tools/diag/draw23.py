"""Random-shape draw 23 (tests/test_gpu_random_shapes.py): the update step in fp32 / fp64, with and
without the CG's residual reorthogonalisation, against the oracle."""
import os, sys
R = os.path.join(os.path.dirname(__file__), "..", "..")
sys.path[:0] = [os.path.join(R, "tests"), os.path.join(R, "trpo-robot-control_amd"), os.path.join(R, "oracle")]
import numpy as np
import cases, oracle, trpo_amd
from trpo_amd import synth
from test_gpu_random_shapes import _draw
seed = int(sys.argv[1]) if len(sys.argv) > 1 else 23
layers, acts, n, std = _draw(seed)
th = synth.make_theta(layers, seed=100 + seed)
obs = synth.make_obs(n, layers[0], seed=200 + seed)
mean, action, adv = synth.make_rollout(layers, acts, th, obs, std, seed=500 + seed)
ref = oracle.update(layers, acts, th, obs, mean, action, adv, std, 0.1)
for prec in ("fp32", "fp64"):
    for ro in ("1", "0"):
        os.environ["TRPO_CG_REORTH"] = ro
        with trpo_amd.Context(layers, acts, th, obs, std, 0.1, precision=prec) as c:
            c.set_rollout(mean, action, adv)
            r = c.update()
            rr, xn, it = c.cg_history()
        print(prec, "reorth", ro, c.kernel_name if False else "", "x relL2 %.3e" % cases.rel_l2(r["x"], ref["x"]),
              "iters", r["cg_iters"], "accepted", r["accepted"], ref["accepted"], flush=True)
