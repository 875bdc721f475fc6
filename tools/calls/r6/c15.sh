# round 6, call 15: the staged-result host calls (download, FVP host call, CG history, the staging wait)
# wait on a stream-written pinned flag instead of a stream sync: the whole GPU suite, then an interleaved
# A/B of the host-visible API calls, before (hw0) and after (hw1)
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
V=trpo-robot-control_amd/lib/variants
tools/gpu_steps.sh \
  700 r6/c15_tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  400 r6/c15_ab.log "for r in 1 2; do for v in hw0 hw1; do echo \"== \$v\"; TRPO_LIB=$V/\$v.so timeout -k 5 120 python tools/host_fvp_call.py || exit \$?; TRPO_LIB=$V/\$v.so timeout -k 5 120 python tools/host_api_timing.py || exit \$?; done; done"
