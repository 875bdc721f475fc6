# round 5, call 21: the GPU suite with every device allocation poisoned first (TRPO_DEBUG_POISON=63), on the
# final kernels (reduce_dots, the split granule exchange, the un-sunk loads)
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
tools/gpu_steps.sh 900 r5/check21_poison_tests.log 'TRPO_DEBUG_POISON=63 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread'
