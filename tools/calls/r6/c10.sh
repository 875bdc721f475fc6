# round 6, call 10: the one-launch baseline evaluate with fence-free (sc1) in-launch hand-offs: the
# baseline / liblbfgs GPU tests, an interleaved A/B of the evaluate and the caller's liblbfgs fit before
# (bl0) and after (bl1), and the host-wait forms (stream write-value and event-query added)
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
V=trpo-robot-control_amd/lib/variants
tools/gpu_steps.sh \
  300 r6/c10_tests.log 'python -u -m pytest tests/test_gpu_baseline.py tests/test_lbfgs_caller.py -m gpu -x -v --timeout 120 --timeout-method thread' \
  400 r6/c10_ab.log "for r in 1 2; do for v in bl0 bl1; do TRPO_LIB=$V/\$v.so timeout -k 5 150 python tools/baseline_eval_timing.py 3000 || exit \$?; done; done" \
  120 r6/c10_host_wait.log 'tools/micro/host_wait'
