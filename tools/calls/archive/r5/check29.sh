# round 5, call 29: GPU suite with the lane-parallel baseline kernel
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
tools/gpu_steps.sh 600 r5/check29_tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread'
