# round-4 final check on the final build: GPU suite, smoke, the driver's bench command, a 4-rank
# one-GPU bench line on the peer exchange (with the N > 1 extras)
export TMPDIR=/tmp
tools/gpu_steps.sh \
  600 final_tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  200 final_smoke.log 'python -u -c "import __graft_entry__ as g; g.smoke()"' \
  300 final_bench.log 'python -u bench.py --steps 20 --warmup 5' \
  400 final_bench4.log 'TRPO_BENCH_DEVICE=0 python -u bench.py --gpus 4 --comm peer --steps 50 --warmup 5'
