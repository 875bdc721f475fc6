# round 6, call 20: kernel trace of the final build's TRPO update (armDOF_0, N = 50k, 20 updates): the
# update's launch structure after the round's host-wait / launch changes
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
tools/gpu_steps.sh \
  200 r6/c20_update_trace.log 'rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6/c20_trace -o run -- python3 tools/update_only.py arm 50000 20'
