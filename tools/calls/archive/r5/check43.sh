# round 5, call 43: the whole GPU suite on the final build
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
tools/gpu_steps.sh \
  600 r5/check43_tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread'
