"""Does freed UNCACHED device memory (hipExtMallocWithFlags(..., hipDeviceMallocUncached), the peer
window's allocation) poison later contexts under the torch-bundled HIP runtime?  Allocates, touches and
frees uncached buffers of the peer window's sizes, then runs the 2x64 single-context FVP against the
oracle.  usage: ... [torch|notorch] [uc|plain]"""
import ctypes as C
import os
import sys

if sys.argv[1] == "torch":
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
kind = sys.argv[2]
layers = [15, 64, 64, 3]
n = 6000
th, obs = synth.make_theta(layers), synth.make_obs(n, layers[0])
std = np.ones(3)
v = synth.make_v(synth.num_params(layers))
zor, _ = oracle.fvp(layers, "lttl", th, obs, std, v)


def single(tag):
    with trpo_amd.Context(layers, "lttl", th, obs, std, 0.1) as one:
        z = one.fvp(v)
        z2 = one.fvp(v)
    print("%s: fvp %.2e again %.2e" % (tag, np.linalg.norm(z - zor) / np.linalg.norm(zor),
                                       np.linalg.norm(z2 - zor) / np.linalg.norm(zor)), flush=True)


single("before")
ptrs = []
for sz in [1 << 20, 1400 << 10, 2 << 20, 4 << 20, 256 << 10, 64 << 10] * 4:
    p = C.c_void_p()
    rc = (hip.hipExtMallocWithFlags(C.byref(p), C.c_size_t(sz), C.c_uint(0x3)) if kind == "uc"
          else hip.hipMalloc(C.byref(p), C.c_size_t(sz)))       # 0x3 = hipDeviceMallocUncached
    if rc == 0:
        hip.hipMemset(p, 0, C.c_size_t(sz))
        ptrs.append(p)
hip.hipDeviceSynchronize()
print("allocated", len(ptrs), kind, flush=True)
for p in ptrs:
    hip.hipFree(p)
hip.hipDeviceSynchronize()
single("after %s alloc/free" % kind)
single("after %s alloc/free, again" % kind)
