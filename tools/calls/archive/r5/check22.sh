# round 5, call 22: kernel traces of the TRPO update (armDOF_0 and 2x64, N = 50k) to look for serialised
# launches and short kernels on its path
export TMPDIR=/tmp
mkdir -p gpurun_out/r5/upd
tools/gpu_steps.sh \
  180 r5/upd/arm.log "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/upd/arm -o run -- python3 tools/update_only.py arm 50000 20" \
  180 r5/upd/w64.log "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/upd/w64 -o run -- python3 tools/update_only.py 2x64 50000 20"
