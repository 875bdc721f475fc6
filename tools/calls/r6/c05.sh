# round 6, call 5: the N > 1 bench path on the final code -- the two-rank GPU bench tests, then a four-rank
# rehearsal of the default command on one GPU (peer exchange headline, RCCL secondary refused on a shared device)
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
tools/gpu_steps.sh \
  300 r6/c05_bench_multi_tests.log 'python -u -m pytest tests/test_gpu_bench_multi.py tests/test_gpu_peer.py -m gpu -x -q --timeout 120 --timeout-method thread' \
  400 r6/c05_bench4.log 'TRPO_BENCH_DEVICE=0 python bench.py --gpus 4 --steps 20 --warmup 5 > gpurun_out/r6/c05_bench_4ranks_1gpu.json'
