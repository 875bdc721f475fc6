"""Child process of tests/test_gpu_peer.py::test_peer_slab_paths_torch_runtime_first: torch is imported
FIRST, so its bundled libamdhip64 (ROCm 7.0) serves libtrpo_mi355x.so as well.  Under that runtime, in rounds
2-4, contexts created after peer-attached contexts had been destroyed computed wrong FVPs; round 5 traced it
to returning the uncached peer window to that runtime (hipFree) and keeps the windows for the life of the
process instead (profiles/r05_peer_diag/).  This script repeats the round-4 reproduction -- the
slab-path peer test (2x64 fp32 and fp64: two in-process ranks through peer windows, FVP and the full
TRPO update against the oracle) twice -- and then checks a fresh single context's FVP.
Exit status 0 = every check passed; prints the runtime in use and one "ok" line per check."""
import os
import sys

import torch  # noqa: F401 -- first, on purpose

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "trpo-robot-control_amd")):
    sys.path.insert(0, p)

import warnings  # noqa: E402

warnings.simplefilter("ignore", RuntimeWarning)
import trpo_amd  # noqa: E402

trpo_amd.lib()
print("runtime:", trpo_amd.runtime_path(), "built-against:", trpo_amd.built_runtime_dir(),
      "same:", trpo_amd.runtime_is_built_one(), flush=True)
import numpy as np  # noqa: E402

import oracle  # noqa: E402
import test_gpu_peer  # noqa: E402
from trpo_amd import synth  # noqa: E402

for r in range(2):
    for kind in ("2x64", "fp64"):
        test_gpu_peer.test_peer_fvp_and_update_slab_paths(kind)
        print("ok", r, kind, flush=True)
layers = [15, 64, 64, 3]
th, obs = synth.make_theta(layers), synth.make_obs(3000, layers[0])
std = np.ones(3)
v = synth.make_v(synth.num_params(layers))
zor, _ = oracle.fvp(layers, "lttl", th, obs, std, v)
with trpo_amd.Context(layers, "lttl", th, obs, std, 0.1) as c:
    for k in range(2):                      # the first FVP (forward pass recomputed) and a cached one
        e = float(np.linalg.norm(c.fvp(v) - zor) / np.linalg.norm(zor))
        assert e <= 1e-5, e
        print("ok single-context fvp %d %.2e" % (k, e), flush=True)
