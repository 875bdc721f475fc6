# round 5, call 39: FVP-call tile order at N = 4 096 (2x64), repeated: forced block-major, the default, forced group-major
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
L=trpo-robot-control_amd/lib/libtrpo_mi355x.so
tools/gpu_steps.sh \
  300 r5/check39_ab_4096.log "SHAPES=2x64 N=4096 ROUNDS=15 python -u tools/ab.py $L:TRPO_COOP_GMAJ=0 $L $L:TRPO_COOP_GMAJ=1" \
  300 r5/check39_ab_4096b.log "SHAPES=2x64 N=4096 ROUNDS=15 python -u tools/ab.py $L $L:TRPO_COOP_GMAJ=0 $L:TRPO_COOP_GMAJ=1" \
  300 r5/check39_ab_3000.log "SHAPES=2x64 N=3000 ROUNDS=11 python -u tools/ab.py $L:TRPO_COOP_GMAJ=0 $L"
