import os, sys, numpy as np
sys.path[:0] = ["tests", "trpo-robot-control_amd", "oracle"]
import cases, trpo_amd, oracle
from trpo_amd import synth
def seg(layers):
    out=[]; pos=0
    for i in range(len(layers)-1):
        out.append(("W%d"%i, pos, pos+layers[i]*layers[i+1])); pos += layers[i]*layers[i+1]
        out.append(("B%d"%i, pos, pos+layers[i+1])); pos += layers[i+1]
    out.append(("LS", pos, pos+layers[-1])); return out
for layers, std in [([15,64,64,3],[1.,1.,1.]), ([15,64,64,3],[0.6065306597126334,0.8,1.3]), ([15,16,16,3],[1.,1.,1.])]:
    P = synth.num_params(layers); th = synth.make_theta(layers); v = synth.make_v(P)
    for n in [4096, 4097, 4080, 1000, 8192, 4096]:
        obs = synth.make_obs(n, 15)
        ref,_ = oracle.fvp(layers, "lttl", th, obs, np.array(std), v)
        with trpo_amd.Context(layers, "lttl", th, obs, np.array(std)) as ctx:
            out = ctx.fvp(v)
            errs = " ".join("%s=%.1e" % (nm, np.linalg.norm(out[a:b]-ref[a:b])/max(1e-300,np.linalg.norm(ref[a:b]))) for nm,a,b in seg(layers))
            print(layers[1], std[0], n, ctx.geometry["blocks"], "rel=%.3e" % cases.rel_l2(out, ref), errs, flush=True)
