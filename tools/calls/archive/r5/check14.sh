# round 5, call 14: the split granule exchange (TRPO_PEER_PROTO=4: W pushing + W polling workgroups):
# one-GPU floor against proto 3 in the same call, then the peer tests under proto 4
export TMPDIR=/tmp
mkdir -p gpurun_out/r5/pf4
tools/gpu_steps.sh \
  240 r5/pf4/p4.log "TRPO_PEER_PROTO=4 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5/pf4/p4 -o run -- python3 tools/peer_floor.py" \
  240 r5/pf4/p3.log "TRPO_PEER_PROTO=3 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5/pf4/p3 -o run -- python3 tools/peer_floor.py" \
  60 r5/pf4/stats.log "python3 tools/peer_floor_stats.py proto4 gpurun_out/r5/pf4/p4 && python3 tools/peer_floor_stats.py proto3 gpurun_out/r5/pf4/p3" \
  400 r5/pf4/peer_tests_p4.log "TRPO_PEER_PROTO=4 python -u -m pytest tests/test_gpu_peer.py tests/test_gpu_bench_multi.py -x -q --timeout 120 --timeout-method thread" \
  300 r5/pf4/bench2ranks_p4.log "TRPO_PEER_PROTO=4 TRPO_BENCH_DEVICE=0 python -u bench.py --gpus 2 --comm peer --steps 100 --warmup 10 --no-extra --no-cpu-baseline" \
  300 r5/pf4/bench2ranks_p3.log "TRPO_PEER_PROTO=3 TRPO_BENCH_DEVICE=0 python -u bench.py --gpus 2 --comm peer --steps 100 --warmup 10 --no-extra --no-cpu-baseline"
