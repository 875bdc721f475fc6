# 2x64: the cooperative kernel vs the one-wave-per-tile kernel (TRPO_COOP=0), interleaved A/B
export TMPDIR=/tmp
L=trpo-robot-control_amd/lib/libtrpo_mi355x.so
tools/gpu_steps.sh \
  300 coop0_50k.log "SHAPES=2x64 ROUNDS=5 python -u tools/ab.py $L $L:TRPO_COOP=0" \
  300 coop0_4k.log "SHAPES=2x64 ROUNDS=5 N=4096 python -u tools/ab.py $L $L:TRPO_COOP=0"
