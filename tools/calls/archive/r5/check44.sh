# round 5, call 44: baseline_lane_kernel with its chains unrolled to 16 (no run-time register indexing)
export TMPDIR=/tmp
mkdir -p gpurun_out/r5/bn3
V=trpo-robot-control_amd/lib/variants/prevlane.so
tools/gpu_steps.sh \
  300 r5/bn3/tests.log "python -u -m pytest tests/test_gpu_baseline.py tests/test_lbfgs_caller.py -x -q --timeout 180 --timeout-method thread" \
  120 r5/bn3/trace_new.log "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/bn3/new -o run -- python3 tools/diag/baseline_n.py" \
  120 r5/bn3/trace_old.log "TRPO_LIB=$V rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/bn3/old -o run -- python3 tools/diag/baseline_n.py" \
  120 r5/bn3/fit_new.log "python3 tests/lbfgs_fit_child.py 5" \
  120 r5/bn3/fit_old.log "TRPO_LIB=$V python3 tests/lbfgs_fit_child.py 5"
