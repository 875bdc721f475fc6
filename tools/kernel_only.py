"""Launch the fused FVP kernel alone (plain FVP mode) REPS times on the bench workload
(armDOF_0, N=50k) -- for rocprofv3 PMC passes."""
import os, sys, numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "trpo-robot-control_amd")]
import trpo_amd
from trpo_amd import synth
L = [int(x) for x in os.environ.get("LAYERS", "15,16,16,3").split(",")]
n = int(os.environ.get("N", "50000"))
th = synth.make_theta(L); P = synth.num_params(L)
with trpo_amd.Context(L, "lttl", th, synth.make_obs(n, L[0]), np.ones(L[-1])) as ctx:
    ctx.upload_v(synth.make_v(P))
    ctx.enqueue_fvp()          # first FVP: writes the forward-activation cache (MODE 0); the rest run MODE 2
    for _ in range(int(os.environ.get("REPS", "50"))):
        ctx.enqueue_fvp_kernel()
    ctx.synchronize()
    print("kernel_ms", ctx.time_ms(0, 20), ctx.kernel_name)
