import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "trpo-robot-control_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

# Load libtrpo_mi355x.so (and with it the system ROCm's libamdhip64.so.7) BEFORE collection imports
# torch (tests/test_dist_gloo.py): torch's wheel bundles its own libamdhip64.so.7, and whichever copy
# is loaded first serves this library for the whole process (see trpo_amd.lib()).
try:
    import trpo_amd
    trpo_amd.lib()
except Exception:           # not built yet: the tests that need it fail loudly on their own
    pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long CPU case (oracle at N=50k)")
