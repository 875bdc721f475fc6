# round-4 check: the GPU suite, the driver's bench command, a two-rank one-GPU bench line on the peer
# exchange (with parity) and smoke()
export TMPDIR=/tmp
tools/gpu_steps.sh \
  600 check_tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  300 check_bench.log 'python -u bench.py --steps 20 --warmup 5' \
  300 check_bench2.log 'TRPO_BENCH_DEVICE=0 python -u bench.py --gpus 2 --comm peer --steps 50 --warmup 5' \
  200 check_smoke.log 'python -u -c "import __graft_entry__ as g; g.smoke()"'
