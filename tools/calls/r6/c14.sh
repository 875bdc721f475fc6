# round 6, call 14: the update's results exported with per-block pinned flags and a host spin (one launch
# and the stream sync fewer), the full-step surrogate summed straight into pinned memory: the whole GPU
# suite, then an interleaved A/B of whole updates, before (up0) and after (up1)
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
V=trpo-robot-control_amd/lib/variants
tools/gpu_steps.sh \
  700 r6/c14_tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  400 r6/c14_ab.log "ROUNDS=7 timeout -k 5 300 python tools/ab_update.py $V/up0.so $V/up1.so"
