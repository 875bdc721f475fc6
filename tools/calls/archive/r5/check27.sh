# round 5, call 27: GPU suite after the generic-kernel changes, the liblbfgs fit child, the driver's bench command
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
tools/gpu_steps.sh \
  600 r5/check27_tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  120 r5/check27_fit.log "python3 tests/lbfgs_fit_child.py 5" \
  300 r5/check27_bench.log 'python -u bench.py --steps 20 --warmup 5'
