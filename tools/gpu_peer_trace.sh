# peer-exchange tests (3 passes) and a kernel trace of two peer ranks on one GPU
export TMPDIR=/tmp
tools/gpu_steps.sh 300 peer.log 'for i in 1 2 3; do python -u -m pytest tests/test_gpu_peer.py -x -q --timeout 120 --timeout-method thread || exit 1; done' \
  200 peer_trace.log 'TRPO_BENCH_DEVICE=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/peer_trace -o run -- python3 bench.py --gpus 2 --comm peer --steps 20 --warmup 3 --no-extra'
