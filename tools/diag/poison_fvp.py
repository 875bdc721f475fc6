"""Uninitialised-memory probe: fill and free many device buffers with 0xFF bytes (NaN in fp32 and fp64)
through the HIP runtime this process uses, so later allocations may reuse poisoned memory, then run each
kernel family's FVP / CG / update against the oracle.  A NaN or a wrong value afterwards means a kernel
read memory the library never wrote.  usage: ... [torch|notorch]"""
import ctypes as C
import os
import sys

if len(sys.argv) > 1 and sys.argv[1] == "torch":
    import torch  # noqa: F401
R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path[:0] = [os.path.join(R, "tests"), os.path.join(R, "trpo-robot-control_amd"), os.path.join(R, "oracle")]
import warnings  # noqa: E402

warnings.simplefilter("ignore", RuntimeWarning)
import numpy as np  # noqa: E402

import trpo_amd  # noqa: E402

trpo_amd.lib()
import oracle  # noqa: E402
from trpo_amd import synth  # noqa: E402

hip = C.CDLL(trpo_amd.runtime_path())
print("runtime", trpo_amd.runtime_path(), flush=True)


def poison():
    ptrs = []
    for sz in [4 << 10, 16 << 10, 64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20] * 4:
        p = C.c_void_p()
        if hip.hipMalloc(C.byref(p), C.c_size_t(sz)) == 0:
            hip.hipMemset(p, 0xFF, C.c_size_t(sz))
            ptrs.append(p)
    hip.hipDeviceSynchronize()
    for p in ptrs:
        hip.hipFree(p)
    hip.hipDeviceSynchronize()


def rel(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


for layers, prec in (([15, 64, 64, 3], "fp32"), ([15, 16, 16, 3], "fp64"), ([15, 16, 16, 3], "fp32"),
                     ([15, 64, 64, 3], "fp64"), ([4, 54, 26, 17, 5], "fp32")):
    acts = "l" + "t" * (len(layers) - 2) + "l"
    n = 6000
    th, obs = synth.make_theta(layers), synth.make_obs(n, layers[0])
    std = np.ones(layers[-1])
    P = synth.num_params(layers)
    v, b = synth.make_v(P), synth.make_b(P)
    zor, _ = oracle.fvp(layers, acts, th, obs, std, v)
    xor = oracle.cg(layers, acts, th, obs, std, b, 10, 0.0)["x"]
    for trial in range(2):
        poison()
        with trpo_amd.Context(layers, acts, th, obs, std, 0.1, precision=prec) as c:
            z = c.fvp(v)
            x = c.cg(b, 10, 0.0)
            z2 = c.fvp(v)
            name = c.kernel_name
        print("%s %s %s trial %d: fvp %.2e cg %.2e fvp#2 %.2e nan %d" % (layers, prec, name, trial, rel(z, zor),
              rel(x, xor), rel(z2, zor), int(np.isnan(z).sum() + np.isnan(x).sum())), flush=True)
