"""Child process of tests/test_gpu_peer.py::test_peer_slab_paths_torch_runtime_first:
torch is imported FIRST, so its bundled libamdhip64 serves libtrpo_mi355x.so as well; then the in-process
two-context peer exchange on the slab paths (the 2x64 cooperative kernel, the fp64 mode) runs exactly as
test_peer_fvp_and_update_slab_paths does.  Under this runtime that test gave rank-equal wrong sums with the
fence-free hand-off; it must pass with the hand-off's release / acquire.
Exit status 0 = every case passed; prints the runtime in use."""
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
import test_gpu_peer  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 1
for r in range(reps):
    for kind in ("2x64", "fp64"):
        test_gpu_peer.test_peer_fvp_and_update_slab_paths(kind)
        print("ok", r, kind, flush=True)
