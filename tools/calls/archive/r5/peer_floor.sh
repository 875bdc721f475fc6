# round 5: the granule exchange with a compile-time world and unconditional poll loads (TRPO_PEER_PROTO=3):
# one-GPU floor (tools/peer_floor.py under a kernel trace) for protos 1 / 2 / 3, then the peer tests and
# the two-rank bench with proto 3
export TMPDIR=/tmp
mkdir -p gpurun_out/r5/pf
tools/gpu_steps.sh \
  240 r5/pf/p3.log "TRPO_PEER_PROTO=3 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5/pf/p3 -o run -- python3 tools/peer_floor.py" \
  240 r5/pf/p1.log "TRPO_PEER_PROTO=1 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5/pf/p1 -o run -- python3 tools/peer_floor.py" \
  240 r5/pf/p2.log "TRPO_PEER_PROTO=2 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5/pf/p2 -o run -- python3 tools/peer_floor.py" \
  60 r5/pf/stats.log "python3 tools/peer_floor_stats.py proto3 gpurun_out/r5/pf/p3 && python3 tools/peer_floor_stats.py proto1 gpurun_out/r5/pf/p1 && python3 tools/peer_floor_stats.py proto2 gpurun_out/r5/pf/p2" \
  400 r5/pf/peer_tests_p3.log "TRPO_PEER_PROTO=3 python -u -m pytest tests/test_gpu_peer.py tests/test_gpu_bench_multi.py -x -q --timeout 120 --timeout-method thread" \
  300 r5/pf/bench2ranks_p3.log "TRPO_PEER_PROTO=3 TRPO_BENCH_DEVICE=0 python -u bench.py --gpus 2 --comm peer --steps 100 --warmup 10 --no-extra --no-cpu-baseline" \
  300 r5/pf/bench2ranks_p1.log "TRPO_PEER_PROTO=1 TRPO_BENCH_DEVICE=0 python -u bench.py --gpus 2 --comm peer --steps 100 --warmup 10 --no-extra --no-cpu-baseline"
