# round 6, call 18: the pushing side's record in the granule exchange -- the whole GPU suite
# (the timeout test asserts the new lines), then the four-rank one-GPU rehearsal of the default N > 1 bench
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
tools/gpu_steps.sh \
  700 r6/c18_tests.log 'python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread' \
  400 r6/c18_bench4.log 'TRPO_BENCH_DEVICE=0 python bench.py --gpus 4 --steps 20 --warmup 5 > gpurun_out/r6/c18_bench_4ranks_1gpu.json'
