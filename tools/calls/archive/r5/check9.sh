# round 5, call 9: the slab reduce and the CG dots in one launch (TRPO_COOP_RDOTS, one rank) and the
# group-major cooperative tile order (TRPO_COOP_GMAJ): GPU suite, then A/B against the knobs off
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
L=trpo-robot-control_amd/lib/libtrpo_mi355x.so
tools/gpu_steps.sh \
  600 r5/check9_tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  300 r5/check9_ab.log "SHAPES=2x64 ROUNDS=9 python -u tools/ab.py $L:TRPO_COOP_RDOTS=0 $L $L:TRPO_COOP_GMAJ=1" \
  300 r5/check9_ab_4096.log "SHAPES=2x64 N=4096 ROUNDS=9 python -u tools/ab.py $L:TRPO_COOP_RDOTS=0 $L $L:TRPO_COOP_GMAJ=1"
