# round 5, call 11: partial dots value-major (cg_axpy's loads coalesced): GPU suite + 2x64 kernel trace;
# the granule exchange with a compile-time world (proto 3) failed the 4-process IPC test once: one run of
# it with the diagnostic build (prints the missing granules on a timeout) and one with proto 2 to compare
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
V=trpo-robot-control_amd/lib/variants/peerdiag.so
tools/gpu_steps.sh \
  600 r5/check11_tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  150 r5/check11_2x64.log 'bash tools/gpu_prof_2x64.sh' \
  200 r5/check11_ipc4_p3diag.log "TRPO_LIB=$V TRPO_PEER_PROTO=3 python -u -m pytest 'tests/test_gpu_peer.py::test_peer_ipc_processes[4]' -x -q --timeout 180 --timeout-method thread" \
  200 r5/check11_ipc4_p2.log "TRPO_PEER_PROTO=2 python -u -m pytest 'tests/test_gpu_peer.py::test_peer_ipc_processes[4]' -x -q --timeout 180 --timeout-method thread"
