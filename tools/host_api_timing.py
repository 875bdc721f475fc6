"""Host-visible wall time of the API calls a trainer makes: Context.fvp (v up, FVP, z down),
Context.cg (b up, CG(10), x down + history), Baseline.evaluate (x up, f/g down) -- armDOF_0."""
import os, sys, time, numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, "trpo-robot-control_amd")]
import trpo_amd
from trpo_amd import synth
L = [15, 16, 16, 3]; P = synth.num_params(L)
for n in (4096, 50000):
    with trpo_amd.Context(L, "lttl", synth.make_theta(L), synth.make_obs(n, 15), np.ones(3), 0.1) as ctx:
        v, b = synth.make_v(P), synth.make_b(P)
        for f, name in ((lambda: ctx.fvp(v), "fvp"), (lambda: ctx.cg(b, 10, 0.0), "cg10"),
                        (lambda: ctx.cg_history(), "cg_history")):
            f(); t0 = time.perf_counter()
            for _ in range(50): f()
            print("n=%d %-10s %.1f us" % (n, name, 1e6 * (time.perf_counter() - t0) / 50), flush=True)
LB = [16, 16, 16, 1]
x, obs, tgt = synth.make_baseline_problem(LB, 20, 150)
with trpo_amd.Baseline(LB, "lttl") as bl:
    bl.set_data(obs, tgt, 20, 150); bl.evaluate(x)
    t0 = time.perf_counter()
    for _ in range(50): bl.evaluate(x)
    print("baseline evaluate N=3000 %.1f us" % (1e6 * (time.perf_counter() - t0) / 50))
