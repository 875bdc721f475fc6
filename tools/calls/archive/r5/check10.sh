# round 5, call 10: group-major cooperative tiles by default on full grids, RS_POS = 16 slab-reduce variant
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
L=trpo-robot-control_amd/lib
tools/gpu_steps.sh \
  600 r5/check10_tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  300 r5/check10_ab.log "SHAPES=2x64 ROUNDS=9 python -u tools/ab.py $L/libtrpo_mi355x.so:TRPO_COOP_GMAJ=0 $L/libtrpo_mi355x.so $L/variants/rs16.so" \
  300 r5/check10_ab_4096.log "SHAPES=2x64 N=4096 ROUNDS=9 python -u tools/ab.py $L/libtrpo_mi355x.so $L/variants/rs16.so $L/variants/rs16.so:TRPO_COOP_GMAJ=1"
