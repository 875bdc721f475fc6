"""Child process of tests/test_gpu_peer.py::test_peer_slab_paths_torch_runtime_first:
torch is imported FIRST, so its bundled libamdhip64 serves libtrpo_mi355x.so as well.  Under that runtime a
peer-attached FVP left later contexts computing wrong FVPs (round-4 bisection), so the library
refuses the peer exchange there: this script checks that opening a peer window fails with an error (no
silent wrong result) and that ordinary single contexts stay correct.  With argument "any" and
TRPO_PEER_ANY_RUNTIME=1 it instead runs the slab-path peer test (the reproduction).
Exit status 0 = every check passed; prints the runtime in use."""
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

if len(sys.argv) > 1 and sys.argv[1] == "any":
    for r in range(2):
        for kind in ("2x64", "fp64"):
            test_gpu_peer.test_peer_fvp_and_update_slab_paths(kind)
            print("ok", r, kind, flush=True)
    raise SystemExit(0)
layers = [15, 64, 64, 3]
th, obs = synth.make_theta(layers), synth.make_obs(3000, layers[0])
std = np.ones(3)
v = synth.make_v(synth.num_params(layers))
zor, _ = oracle.fvp(layers, "lttl", th, obs, std, v)
refused = 0
for r in range(2):
    with trpo_amd.Context(layers, "lttl", th, obs, std, 0.1) as c:
        e = float(np.linalg.norm(c.fvp(v) - zor) / np.linalg.norm(zor))
        assert e <= 1e-5, e
        try:
            c.peer_handle()
        except trpo_amd.TRPOError as err:
            refused += 1
            print("refused:", err, flush=True)
    print("ok", r, "single-context fvp %.2e" % e, flush=True)
assert refused == 2 or trpo_amd.runtime_is_built_one(), refused
