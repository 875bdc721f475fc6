# round 6, call 9: the one-launch baseline evaluate (theta by value, in-launch slab sum, pinned-memory
# hand-off): the baseline / liblbfgs GPU tests, then an interleaved A/B of the evaluate and the caller's
# liblbfgs fit, before (bl0) and after (bl1)
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
V=trpo-robot-control_amd/lib/variants
tools/gpu_steps.sh \
  300 r6/c09_tests.log 'python -u -m pytest tests/test_gpu_baseline.py tests/test_lbfgs_caller.py -m gpu -x -v --timeout 120 --timeout-method thread' \
  400 r6/c09_ab.log "for r in 1 2; do for v in bl0 bl1; do TRPO_LIB=$V/\$v.so timeout -k 5 150 python tools/baseline_eval_timing.py 3000 || exit \$?; done; done"
