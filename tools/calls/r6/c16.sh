# round 6, call 16: the final build (update / host-call flag waits, moving-offset guards and their tests) --
# the whole GPU suite, smoke, and the driver's bench command
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
tools/gpu_steps.sh \
  700 r6/c16_tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  120 r6/c16_smoke.log 'python -c "import __graft_entry__ as g; g.smoke()"' \
  600 r6/c16_bench.log 'python bench.py --steps 20 --warmup 5 > gpurun_out/r6/c16_bench_steps20_warmup5.json'
