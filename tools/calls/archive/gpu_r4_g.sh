# round 4 validation: the GPU suite, the driver's bench command twice, and kernel traces of the headline
# alone and of the whole bench command
export TMPDIR=/tmp
tools/gpu_steps.sh \
  600 tests.log 'TRPO_TIMING_OUT=gpurun_out/r04_lbfgs_fit_timing.json python -u -m pytest tests -m gpu -v -s --timeout 120 --timeout-method thread' \
  300 bench_driver1.log 'python -u bench.py --steps 20 --warmup 5' \
  300 bench_driver2.log 'python -u bench.py --steps 20 --warmup 5' \
  200 prof_head.log 'rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r04_head -o run -- python3 bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline' \
  300 prof_full.log 'rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r04_full -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline'
