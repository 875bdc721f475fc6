# floor of one peer exchange on ONE GPU (tools/peer_floor.py under a kernel trace) for the three
# exchange forms (TRPO_PEER_PROTO 2 tagged granules / 1 flag + batched loads / 0 round-3 loops); then
# the peer tests and the two-rank bench line per form
export TMPDIR=/tmp
mkdir -p gpurun_out/peer_floor
tools/gpu_steps.sh \
  240 peer_floor/p2.log "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/peer_floor/p2 -o run -- python3 tools/peer_floor.py" \
  240 peer_floor/p1.log "TRPO_PEER_PROTO=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/peer_floor/p1 -o run -- python3 tools/peer_floor.py" \
  240 peer_floor/p0.log "TRPO_PEER_PROTO=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/peer_floor/p0 -o run -- python3 tools/peer_floor.py" \
  400 peer_tests.log "python -u -m pytest tests/test_gpu_peer.py tests/test_gpu_bench_multi.py -x -q --timeout 120 --timeout-method thread" \
  300 bench2ranks_p2.log "TRPO_BENCH_DEVICE=0 python -u bench.py --gpus 2 --comm peer --steps 100 --warmup 10 --no-extra" \
  300 bench2ranks_p1.log "TRPO_PEER_PROTO=1 TRPO_BENCH_DEVICE=0 python -u bench.py --gpus 2 --comm peer --steps 100 --warmup 10 --no-extra --no-cpu-baseline" \
  300 bench2ranks_p0.log "TRPO_PEER_PROTO=0 TRPO_BENCH_DEVICE=0 python -u bench.py --gpus 2 --comm peer --steps 100 --warmup 10 --no-extra --no-cpu-baseline"
