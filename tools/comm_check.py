"""CG time with and without a one-rank RCCL communicator attached (the per-FVP all-reduce cost)."""
import os, sys
sys.path[:0] = ["trpo-robot-control_amd"]
import numpy as np, trpo_amd
from trpo_amd import synth
L = [15, 16, 16, 3]
with trpo_amd.Context(L, "lttl", synth.make_theta(L), synth.make_obs(50000, 15), np.ones(3)) as ctx:
    ctx.upload_b(synth.make_b(ctx.P))
    t0 = ctx.time_ms(2, 20, 10, 0.0)
    ctx.attach_comm(0, 1, trpo_amd.unique_id())
    t1 = ctx.time_ms(2, 20, 10, 0.0)
    print("cg ms plain %.4f  with 1-rank RCCL %.4f" % (t0, t1), flush=True)
