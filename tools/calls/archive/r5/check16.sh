# round 5, call 16: the split granule exchange (proto 4) as the default: GPU suite, the two-rank peer bench
# (default) and its flag-form twin
export TMPDIR=/tmp
mkdir -p gpurun_out/r5/pf6
tools/gpu_steps.sh \
  600 r5/check16_tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  300 r5/pf6/bench2ranks_p4.log "TRPO_BENCH_DEVICE=0 python -u bench.py --gpus 2 --comm peer --steps 100 --warmup 10 --no-extra --no-cpu-baseline" \
  300 r5/pf6/bench2ranks_p1.log "TRPO_PEER_PROTO=1 TRPO_BENCH_DEVICE=0 python -u bench.py --gpus 2 --comm peer --steps 100 --warmup 10 --no-extra --no-cpu-baseline"
