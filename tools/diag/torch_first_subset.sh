#!/bin/bash
# GPU test files up to test_gpu_peer.py with torch (and so torch's bundled HIP runtime) loaded first,
# as pytest's collection of tests/test_dist_gloo.py does in the full suite.
timeout -k 10 300 python -u -c "import torch, pytest, sys; sys.exit(pytest.main(['tests/test_gpu_baseline.py', 'tests/test_gpu_c_caller.py', 'tests/test_gpu_comm.py', 'tests/test_gpu_fp64.py', 'tests/test_gpu_parity.py', 'tests/test_gpu_peer.py', '-x', '-q', '--timeout', '120', '--timeout-method', 'thread']))"
