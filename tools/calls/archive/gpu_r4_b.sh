# round 4: the driver's bench command, the full GPU suite, the torch-first peer test replayed, and a
# kernel trace of the bench command
export TMPDIR=/tmp
tools/gpu_steps.sh \
  300 bench_driver.log 'python -u bench.py --steps 20 --warmup 5' \
  600 tests.log 'python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread' \
  200 torchfirst_fence2.log 'python -u tests/peer_torch_first.py 2' \
  300 prof.log 'rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r04 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline'
