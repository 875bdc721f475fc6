"""Kernel-time sweep over N and grid size (env TRPO_FVP_BLOCKS), both shapes."""
import os, sys, json, numpy as np
sys.path[:0] = ["trpo-robot-control_amd"]
import trpo_amd
from trpo_amd import synth
def fps(L):
    S = sum(L[i]*L[i+1] for i in range(len(L)-1)); return 2*(5*S-2*L[0]*L[1]) + 7*sum(L[1:-1]) + 2*L[-1]
def fps_cached(L):   # the forward-activation-cache FVP (bench.py flops_per_sample_cached)
    S = sum(L[i]*L[i+1] for i in range(len(L)-1)); return 2*(4*S-2*L[0]*L[1]) + 7*sum(L[1:-1]) + 2*L[-1]
shapes = {"arm": [15,16,16,3], "2x64": [15,64,64,3]}
Ns = [int(x) for x in os.environ.get("NS", "16,4096,50000,500000").split(",")]
grids = [int(x) for x in os.environ.get("GRIDS", "0").split(",")]
for name, L in shapes.items():
    th = synth.make_theta(L); P = synth.num_params(L); v = synth.make_v(P); b = synth.make_b(P)
    for n in Ns:
        obs = synth.make_obs(n, 15)
        for g in grids:
            if g: os.environ["TRPO_FVP_BLOCKS"] = str(g)
            else: os.environ.pop("TRPO_FVP_BLOCKS", None)
            with trpo_amd.Context(L, "lttl", th, obs, np.ones(3)) as ctx:
                ctx.upload_v(v); ctx.upload_b(b)
                k = ctx.time_ms(0, 100); f = ctx.time_ms(1, 100); c = ctx.time_ms(2, 20, 10, 0.0)
                print(json.dumps(dict(shape=name, n=n, grid=ctx.geometry["blocks"], kernel_us=k*1e3, fvp_us=f*1e3,
                      cg10_us=c*1e3, tflops_cached=fps_cached(L)*n/(k*1e-3)/1e12,
                      tflops_recompute_equiv=fps(L)*n/(k*1e-3)/1e12)), flush=True)
