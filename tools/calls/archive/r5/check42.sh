# round 5, call 42: kernel trace of the armDOF_0 TRPO update (where its non-CG time goes)
export TMPDIR=/tmp
mkdir -p gpurun_out/r5/upd
tools/gpu_steps.sh \
  200 r5/upd/trace.log "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/upd -o run -- python3 tools/update_only.py arm 50000 20"
