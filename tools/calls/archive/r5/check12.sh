# round 5, call 12: block-major vs value-major partial dots (A/B), and the proto-3 exchange with a poll
# backoff: its floor, then the peer tests + two-rank bench tests under it (once)
export TMPDIR=/tmp
mkdir -p gpurun_out/r5/pf2
L=trpo-robot-control_amd/lib
tools/gpu_steps.sh \
  300 r5/check12_ab.log "SHAPES=2x64 ROUNDS=9 python -u tools/ab.py $L/libtrpo_mi355x.so $L/variants/vmaj.so" \
  240 r5/pf2/p3.log "TRPO_PEER_PROTO=3 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5/pf2/p3 -o run -- python3 tools/peer_floor.py" \
  60 r5/pf2/stats.log "python3 tools/peer_floor_stats.py proto3 gpurun_out/r5/pf2/p3" \
  400 r5/pf2/peer_tests_p3.log "TRPO_PEER_PROTO=3 python -u -m pytest tests/test_gpu_peer.py tests/test_gpu_bench_multi.py -x -q --timeout 120 --timeout-method thread"
