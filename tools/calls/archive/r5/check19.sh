# round 5, call 19: group-major cooperative tiles also at <= cus / 2 tiles: GPU suite
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
tools/gpu_steps.sh 600 r5/check19_tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread'
