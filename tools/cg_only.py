"""Run the armDOF_0 (and 2x64) 10-iteration CG graph back to back (for rocprofv3)."""
import os, sys, numpy as np
sys.path[:0] = ["trpo-robot-control_amd"]
import trpo_amd
from trpo_amd import synth
for L in ([15,16,16,3], [15,64,64,3]):
    th = synth.make_theta(L); P = synth.num_params(L)
    with trpo_amd.Context(L, "lttl", th, synth.make_obs(50000, 15), np.ones(3)) as ctx:
        ctx.upload_b(synth.make_b(P))
        print(L, "cg10_us", ctx.time_ms(2, int(os.environ.get("REPS", "50")), 10, 0.0) * 1e3, flush=True)
