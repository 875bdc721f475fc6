"""Host-visible wall time of Context.fvp (v up, FVP, z down) for the C2 shape (2x64, N = 4096) and
armDOF_0 at N = 50k.  usage: TRPO_LIB=<lib.so> python tools/host_fvp_call.py"""
import os, sys, time, numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, "trpo-robot-control_amd")]
import trpo_amd
from trpo_amd import synth
for L, n in (([15, 64, 64, 3], 4096), ([15, 64, 64, 3], 50000), ([15, 16, 16, 3], 50000)):
    P = synth.num_params(L)
    with trpo_amd.Context(L, "lttl", synth.make_theta(L), synth.make_obs(n, 15), np.ones(3), 0.1) as ctx:
        v = synth.make_v(P)
        z0 = ctx.fvp(v)
        meds = []
        for _ in range(5):
            t0 = time.perf_counter()
            for _ in range(200): z = ctx.fvp(v)
            meds.append(1e6 * (time.perf_counter() - t0) / 200)
        assert np.array_equal(z, z0)
        print("%s n=%d fvp call %.2f us (min of 5 x 200), %s" % ("x".join(map(str, L)), n, min(meds), ctx.kernel_name),
              flush=True)
