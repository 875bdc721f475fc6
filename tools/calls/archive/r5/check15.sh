# round 5, call 15: the granule kernels with loads-first ordering (window pointers by value, counter / done
# loaded with the first loads, the error word only off the fast path): floors of protos 4 / 3 / 1 in one
# call, then the peer tests under protos 4 and 3
export TMPDIR=/tmp
mkdir -p gpurun_out/r5/pf5
tools/gpu_steps.sh \
  240 r5/pf5/p4.log "TRPO_PEER_PROTO=4 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5/pf5/p4 -o run -- python3 tools/peer_floor.py" \
  240 r5/pf5/p3.log "TRPO_PEER_PROTO=3 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5/pf5/p3 -o run -- python3 tools/peer_floor.py" \
  240 r5/pf5/p1.log "TRPO_PEER_PROTO=1 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5/pf5/p1 -o run -- python3 tools/peer_floor.py" \
  60 r5/pf5/stats.log "python3 tools/peer_floor_stats.py proto4 gpurun_out/r5/pf5/p4 && python3 tools/peer_floor_stats.py proto3 gpurun_out/r5/pf5/p3 && python3 tools/peer_floor_stats.py proto1 gpurun_out/r5/pf5/p1" \
  400 r5/pf5/peer_tests_p4.log "TRPO_PEER_PROTO=4 python -u -m pytest tests/test_gpu_peer.py tests/test_gpu_bench_multi.py -x -q --timeout 120 --timeout-method thread" \
  400 r5/pf5/peer_tests_p3.log "TRPO_PEER_PROTO=3 python -u -m pytest tests/test_gpu_peer.py tests/test_gpu_bench_multi.py -x -q --timeout 120 --timeout-method thread"
