# round 5, call 28: the lane-parallel baseline objective kernel (baseline_lane_kernel): its tests against the
# oracle and the reference fit, then evaluate timing / fit timing against the one-lane kernel
export TMPDIR=/tmp
mkdir -p gpurun_out/r5/bl
tools/gpu_steps.sh \
  300 r5/bl/tests.log "python -u -m pytest tests/test_gpu_baseline.py tests/test_lbfgs_caller.py -x -q --timeout 180 --timeout-method thread" \
  180 r5/bl/bn_lane.log "rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5/bl/tr -o run -- python3 tools/diag/baseline_n.py" \
  120 r5/bl/bn_one.log "TRPO_BASELINE_LANE=0 python3 tools/diag/baseline_n.py" \
  120 r5/bl/fit_lane.log "python3 tests/lbfgs_fit_child.py 5" \
  120 r5/bl/fit_one.log "TRPO_BASELINE_LANE=0 python3 tests/lbfgs_fit_child.py 5"
