# round 5, call 18: group-major tiles forced at 2x64 N = 4 096 again, now that the slab reduce's first
# round loads every partial slot unconditionally (the reduce cost no longer halves with half the partials)
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
L=trpo-robot-control_amd/lib/libtrpo_mi355x.so
tools/gpu_steps.sh \
  300 r5/check18_ab_4096.log "SHAPES=2x64 N=4096 ROUNDS=11 python -u tools/ab.py $L $L:TRPO_COOP_GMAJ=1" \
  300 r5/check18_ab_8192.log "SHAPES=2x64 N=8192 ROUNDS=7 python -u tools/ab.py $L $L:TRPO_COOP_GMAJ=1" \
  300 r5/check18_ab_2048.log "SHAPES=2x64 N=2048 ROUNDS=7 python -u tools/ab.py $L $L:TRPO_COOP_GMAJ=1"
