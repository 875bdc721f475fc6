# round 5, call 7: the direction pack for standalone cooperative FVPs (packed at upload) and the compact
# fp32 slab layout: GPU suite, A/B (pre-round-5 build / no compact slab / PK off / all on), coop stamps
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
L=trpo-robot-control_amd/lib
tools/gpu_steps.sh \
  600 r5/check7_tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  300 r5/check7_ab.log "SHAPES=2x64 ROUNDS=9 python -u tools/ab.py $L/variants/pre.so $L/variants/nocompact.so $L/libtrpo_mi355x.so:TRPO_COOP_PK=0 $L/libtrpo_mi355x.so" \
  300 r5/check7_ab_4096.log "SHAPES=2x64 N=4096 ROUNDS=9 python -u tools/ab.py $L/variants/pre.so $L/variants/nocompact.so $L/libtrpo_mi355x.so:TRPO_COOP_PK=0 $L/libtrpo_mi355x.so" \
  120 r5/check7_stamps.log 'python -u tools/stamps_coop.py 4096 50000'
