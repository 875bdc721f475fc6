"""Forward-cache bitwise check per activation string: FVP #1 (MODE 0, writes the cache) vs FVP #2 (MODE 2)."""
import os, sys, numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "trpo-robot-control_amd")]
import trpo_amd
from trpo_amd import synth
L = [15, 16, 16, 3]
th, obs = synth.make_theta(L), synth.make_obs(777, 15)
v = synth.make_v(synth.num_params(L))
for acf in sys.argv[1:]:
    with trpo_amd.Context(L, acf, th, obs, np.array([0.7, 1.0, 1.4]), 0.1) as ctx:
        a = ctx.fvp(v); b = ctx.fvp(v)
        print(acf, ctx.kernel_name, "maxrel %.3e" % (np.max(np.abs(a - b)) / np.max(np.abs(a))), flush=True)
