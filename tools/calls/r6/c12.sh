# round 6, call 12: the evaluate with one sample per group and the data comparison overlapped with the
# device (bl4 = the product build): baseline / liblbfgs / C-caller GPU tests, then an interleaved A/B
# against the round-5 form (bl0), and the kernel trace of the evaluate loop
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
V=trpo-robot-control_amd/lib/variants
tools/gpu_steps.sh \
  300 r6/c12_tests.log 'python -u -m pytest tests/test_gpu_baseline.py tests/test_lbfgs_caller.py tests/test_gpu_c_caller.py -m gpu -x -v --timeout 120 --timeout-method thread' \
  400 r6/c12_ab.log "for r in 1 2; do for v in bl0 bl4; do TRPO_LIB=$V/\$v.so timeout -k 5 150 python tools/baseline_eval_timing.py 3000 || exit \$?; done; done" \
  200 r6/c12_eval_trace.log 'rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6/c12_trace -o run -- python3 tools/baseline_eval_timing.py 500'
