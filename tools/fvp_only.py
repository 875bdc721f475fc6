"""Run R full FVP calls (slot V -> Z: the trpo_dev_fvp launch sequence) for kernel-trace timelines.
usage: python tools/fvp_only.py [arm|2x64] [n] [reps]"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "trpo-robot-control_amd")]
import trpo_amd
from trpo_amd import synth
shape = sys.argv[1] if len(sys.argv) > 1 else "2x64"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
L = [15, 16, 16, 3] if shape == "arm" else [15, 64, 64, 3]
with trpo_amd.Context(L, "lttl", synth.make_theta(L), synth.make_obs(n, 15), np.ones(3)) as ctx:
    ctx.upload_v(synth.make_v(ctx.P))
    for _ in range(reps):
        ctx.enqueue_fvp()
    ctx.synchronize()
    print(ctx.kernel_name, "fvp ms", ctx.time_ms(1, 50))
