# the 16-byte-store / transposed-read tile transposes in the cooperative kernel's RGW2 and RGW0 too
# (this build) vs lib/variants/scr0.so (scratch transposes in both kernels): 2x64 A/B, then the suite
export TMPDIR=/tmp
L=trpo-robot-control_amd/lib/libtrpo_mi355x.so
V=trpo-robot-control_amd/lib/variants
mkdir -p gpurun_out/scrxt2
tools/gpu_steps.sh \
  300 scrxt2/ab50k.log "SHAPES=2x64 ROUNDS=7 python -u tools/ab.py $L $V/scr0.so" \
  300 scrxt2/ab4k.log "SHAPES=2x64 ROUNDS=7 N=4096 python -u tools/ab.py $L $V/scr0.so" \
  600 scrxt2/tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread'
