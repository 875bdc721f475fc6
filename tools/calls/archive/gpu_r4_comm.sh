# round 4: the peer hand-off under torch's runtime (fence off = diagnosis, fence on = fix), the GPU
# suite, and the driver's bench command
export TMPDIR=/tmp
tools/gpu_steps.sh \
  200 torchfirst_nofence.log 'TRPO_PEER_FENCE=0 python -u tests/peer_torch_first.py 3' \
  200 torchfirst_fence.log 'python -u tests/peer_torch_first.py 3' \
  600 tests.log 'python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread' \
  300 bench_driver.log 'python -u bench.py --steps 20 --warmup 5'
