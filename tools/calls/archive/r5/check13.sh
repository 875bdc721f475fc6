# round 5, call 13: the proto-3 granule exchange as the default: GPU suite, one-GPU floor of protos 3 and 1
# in the same call, the two-rank peer bench (default form) and its flag-form twin
export TMPDIR=/tmp
mkdir -p gpurun_out/r5/pf3
tools/gpu_steps.sh \
  600 r5/check13_tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  240 r5/pf3/p3.log "rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5/pf3/p3 -o run -- python3 tools/peer_floor.py" \
  240 r5/pf3/p1.log "TRPO_PEER_PROTO=1 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5/pf3/p1 -o run -- python3 tools/peer_floor.py" \
  60 r5/pf3/stats.log "python3 tools/peer_floor_stats.py proto3 gpurun_out/r5/pf3/p3 && python3 tools/peer_floor_stats.py proto1 gpurun_out/r5/pf3/p1" \
  300 r5/pf3/bench2ranks_p3.log "TRPO_BENCH_DEVICE=0 python -u bench.py --gpus 2 --comm peer --steps 100 --warmup 10 --no-extra --no-cpu-baseline" \
  300 r5/pf3/bench2ranks_p1.log "TRPO_PEER_PROTO=1 TRPO_BENCH_DEVICE=0 python -u bench.py --gpus 2 --comm peer --steps 100 --warmup 10 --no-extra --no-cpu-baseline"
