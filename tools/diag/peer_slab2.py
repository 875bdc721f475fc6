"""Diagnostic: the slab-path peer FVP with device memory pre-dirtied (hipMalloc/hipMemset/hipFree of a
large block before the contexts are created), and the same with fresh memory."""
import ctypes as C, os, sys
if os.environ.get("DIAG_TORCH"):
    import torch  # noqa: F401  (as pytest collection of test_dist_gloo does)
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "..", "tests"),
                os.path.join(os.path.dirname(__file__), "..", "..", "trpo-robot-control_amd"),
                os.path.join(os.path.dirname(__file__), "..", "..", "oracle")]
import numpy as np
import cases, oracle, trpo_amd
from trpo_amd import synth
from test_gpu_peer import run_peer_ranks

hip = C.CDLL("libamdhip64.so")
trpo_amd.lib()
print(sorted({l.split()[-1] for l in open("/proc/self/maps") if "amdhip64" in l or "rccl" in l or "hsa-runtime" in l}))
def dirty(nbytes, byte):
    p = C.c_void_p()
    assert hip.hipMalloc(C.byref(p), C.c_size_t(nbytes)) == 0
    assert hip.hipMemset(p, byte, C.c_size_t(nbytes)) == 0
    assert hip.hipDeviceSynchronize() == 0
    assert hip.hipFree(p) == 0

layers = [15, 64, 64, 3]
n = 6000
th, obs = synth.make_theta(layers), synth.make_obs(n, layers[0])
std = np.ones(3)
P = synth.num_params(layers)
v = synth.make_v(P)
mean, action, adv = synth.make_rollout(layers, "lttl", th, obs, std)
zor, _ = oracle.fvp(layers, "lttl", th, obs, std, v)
bounds = [(0, 2500), (2500, n)]
for trial in range(6):
    if trial % 2: dirty(1 << 30, 0x3f)
    ctxs = [trpo_amd.Context(layers, "lttl", th, obs[lo:hi], std, 0.1) for lo, hi in bounds]
    for ctx, (lo, hi) in zip(ctxs, bounds):
        ctx.set_rollout(mean[lo:hi], action[lo:hi], adv[lo:hi])
    try:
        res = run_peer_ranks(ctxs, lambda c, r: (c.fvp(v), c.update(), c.fvp(v)),
                             warm=lambda c: (c.fvp(v), c.update()))
    finally:
        for c in ctxs: c.close()
    z1, z2 = res[0][0], res[0][2]
    bad = np.nonzero(np.abs(z1 - zor) > 1e-4 * np.abs(zor) + 1e-9)[0]
    print("trial", trial, "dirty" if trial % 2 else "clean", "fvp1", cases.rel_l2(z1, zor), "fvp2",
          cases.rel_l2(z2, zor), "nbad", len(bad), "first", bad[:10], "last", bad[-5:] if len(bad) else [],
          flush=True)
