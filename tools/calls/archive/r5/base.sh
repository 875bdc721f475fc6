# round-5 baseline on the round-4 build: GPU suite, the driver's bench command
export TMPDIR=/tmp
tools/gpu_steps.sh \
  600 r5_base_tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  300 r5_base_bench.log 'python -u bench.py --steps 20 --warmup 5'
