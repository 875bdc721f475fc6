# round 5, call 6: GPU suite (torch-first peer test now asserts correct results), the pre-packed direction
# of the distributed 2x64 CG step (TRPO_COOP_PK) A/B, and the coop prologue/epilogue stamps
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
L=trpo-robot-control_amd/lib
tools/gpu_steps.sh \
  600 r5/check6_tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  300 r5/check6_ab_pk.log "SHAPES=2x64 ROUNDS=9 python -u tools/ab.py $L/libtrpo_mi355x.so:TRPO_COOP_PK=0 $L/libtrpo_mi355x.so" \
  300 r5/check6_ab_pk_4096.log "SHAPES=2x64 N=4096 ROUNDS=9 python -u tools/ab.py $L/libtrpo_mi355x.so:TRPO_COOP_PK=0 $L/libtrpo_mi355x.so" \
  120 r5/check6_stamps.log 'python -u tools/stamps_coop.py 4096 50000'
