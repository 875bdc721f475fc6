# round 5, call 26: the generic fp64 kernels (baseline evaluate, generic policy gradient and surrogate)
# specialised on LDS residency (no flat accesses): baseline evaluate vs N, the liblbfgs fit child, and the
# baseline / update / surrogate GPU tests
export TMPDIR=/tmp
mkdir -p gpurun_out/r5/bn2
tools/gpu_steps.sh \
  180 r5/bn2/bn.log "rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5/bn2/tr -o run -- python3 tools/diag/baseline_n.py" \
  120 r5/bn2/fit.log "python3 tests/lbfgs_fit_child.py 5" \
  600 r5/bn2/tests.log "python -u -m pytest tests/test_gpu_baseline.py tests/test_lbfgs_caller.py tests/test_gpu_update.py tests/test_gpu_surrogate.py tests/test_gpu_random_shapes.py tests/test_gpu_fp64.py -x -q --timeout 180 --timeout-method thread"
