# round 4 final-form validation: GPU suite, the driver's bench command twice, the round profile
# (kernel trace, PMC traffic, SQ counters, full bench with the new traffic)
export TMPDIR=/tmp
tools/gpu_steps.sh \
  600 tests.log 'TRPO_TIMING_OUT=gpurun_out/r04_lbfgs_fit_timing.json python -u -m pytest tests -m gpu -v -s --timeout 120 --timeout-method thread' \
  300 bench_driver1.log 'python -u bench.py --steps 20 --warmup 5' \
  300 bench_driver2.log 'python -u bench.py --steps 20 --warmup 5' && \
timeout -k 10 1000 bash tools/profile_round.sh r04
