# round 6, call 11: the two-launch baseline evaluate (theta by value, slab sum into pinned memory with
# per-block flags, host spin): the baseline / liblbfgs GPU tests, then an interleaved A/B of the evaluate
# and the caller's liblbfgs fit: round-5 form (bl0), this form at 2 and 1 samples per 16-lane group (bl3)
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
V=trpo-robot-control_amd/lib/variants
tools/gpu_steps.sh \
  300 r6/c11_tests.log 'python -u -m pytest tests/test_gpu_baseline.py tests/test_lbfgs_caller.py -m gpu -x -v --timeout 120 --timeout-method thread' \
  500 r6/c11_ab.log "for r in 1 2; do for v in bl0:2 bl3:2 bl3:1; do TRPO_BASELINE_SPG=\${v#*:} TRPO_LIB=$V/\${v%:*}.so timeout -k 5 150 python tools/baseline_eval_timing.py 3000 || exit \$?; echo \"(spg \${v#*:})\"; done; done"
