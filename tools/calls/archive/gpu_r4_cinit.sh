# 2x64: the distributed CG start fused into the first FVP launch (default) vs the cg_init launch
# (TRPO_COOP_CINIT=0): interleaved A/B at 50k and 4096, then the GPU suite
export TMPDIR=/tmp
L=trpo-robot-control_amd/lib/libtrpo_mi355x.so
mkdir -p gpurun_out/cinit
tools/gpu_steps.sh \
  300 cinit/ab50k.log "SHAPES=2x64 ROUNDS=7 python -u tools/ab.py $L $L:TRPO_COOP_CINIT=0" \
  300 cinit/ab4k.log "SHAPES=2x64 ROUNDS=7 N=4096 python -u tools/ab.py $L $L:TRPO_COOP_CINIT=0" \
  600 cinit/tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread'
