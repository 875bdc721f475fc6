"""Run R CG(10) solves (armDOF_0 or 2x64, N samples) for kernel-trace timelines.
usage: python tools/cg_only.py [arm|2x64] [n] [reps]   (env TRPO_* knobs apply)"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "trpo-robot-control_amd")]
import trpo_amd
from trpo_amd import synth
shape = sys.argv[1] if len(sys.argv) > 1 else "arm"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 50000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
L = [15, 16, 16, 3] if shape == "arm" else [15, 64, 64, 3]
with trpo_amd.Context(L, "lttl", synth.make_theta(L), synth.make_obs(n, 15), np.ones(3)) as ctx:
    ctx.upload_b(synth.make_b(ctx.P))
    for _ in range(reps):
        ctx.enqueue_cg(10, 0.0)
    ctx.synchronize()
    print(ctx.kernel_name, "cg ms", ctx.time_ms(2, 50, 10, 0.0))
