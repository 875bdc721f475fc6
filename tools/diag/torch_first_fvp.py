"""Which step of a single-context slab-path FVP goes wrong when torch's bundled HIP runtime serves the
library (tests/peer_torch_first.py found the single context 2e-3 off the oracle, the 2-rank peer result
right)?  usage: python tools/diag/torch_first_fvp.py [torch|notorch]"""
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

print("runtime", trpo_amd.runtime_path(), "built-one", trpo_amd.runtime_is_built_one(), flush=True)


def rel(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


for layers, prec, env in (([15, 64, 64, 3], "fp32", {}), ([15, 64, 64, 3], "fp32", {"TRPO_YCACHE": "0"}),
                          ([15, 16, 16, 3], "fp64", {}), ([15, 16, 16, 3], "fp32", {"TRPO_ATOMIC": "0"}),
                          ([15, 16, 16, 3], "fp32", {})):
    for k, v_ in env.items():
        os.environ[k] = v_
    n = 6000
    th, obs = synth.make_theta(layers), synth.make_obs(n, layers[0])
    std = np.ones(layers[-1])
    v = synth.make_v(synth.num_params(layers))
    zor, _ = oracle.fvp(layers, "lttl", th, obs, std, v)
    with trpo_amd.Context(layers, "lttl", th, obs, std, 0.1, precision=prec) as c:
        z1 = c.fvp(v)
        zd1 = c.download_z()
        z2 = c.fvp(v)
        zd2 = c.download_z()
        c.upload_v(v)
        c.enqueue_fvp()
        c.synchronize()
        zd3 = c.download_z()
        name = c.kernel_name
    bad = np.nonzero(np.abs(z1 - zor) > 1e-5 * np.abs(zor).max())[0]
    print("%s %s %s %s: fvp#1 host %.2e dev %.2e | fvp#2 host %.2e dev %.2e | enqueue_fvp dev %.2e | bad %d %s"
          % (layers, prec, env, name, rel(z1, zor), rel(zd1, zor), rel(z2, zor), rel(zd2, zor), rel(zd3, zor),
             len(bad), bad[:12].tolist()), flush=True)
    for k in env:
        os.environ.pop(k)
