# cooperative kernel: RGW1 operands read transposed from the padded exchange rows (TRPO_COOP_XT=1,
# this build) vs the scratch transposes (lib/variants/xt0.so): interleaved A/B, kernel trace, GPU suite
export TMPDIR=/tmp
L=trpo-robot-control_amd/lib/libtrpo_mi355x.so
V=trpo-robot-control_amd/lib/variants
mkdir -p gpurun_out/xt
tools/gpu_steps.sh \
  300 xt/ab50k.log "SHAPES=2x64 ROUNDS=7 python -u tools/ab.py $L $V/xt0.so" \
  300 xt/ab4k.log "SHAPES=2x64 ROUNDS=7 N=4096 python -u tools/ab.py $L $V/xt0.so" \
  200 xt/trace.log "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/xt/trace -o run -- python3 tools/cg_only.py 2x64 50000 20" \
  600 xt/tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread'
