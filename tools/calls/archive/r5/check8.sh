# round 5, call 8: RGW2 of the narrow-output cooperative kernel on the VALU (TRPO_COOP_NOV): GPU suite and
# A/B against the previous form (nov0) and the pre-round-5 build; FVP rows now time the packed direction
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
L=trpo-robot-control_amd/lib
tools/gpu_steps.sh \
  600 r5/check8_tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  300 r5/check8_ab.log "SHAPES=2x64 ROUNDS=9 python -u tools/ab.py $L/variants/pre.so $L/variants/nov0.so $L/libtrpo_mi355x.so" \
  300 r5/check8_ab_4096.log "SHAPES=2x64 N=4096 ROUNDS=9 python -u tools/ab.py $L/variants/pre.so $L/variants/nov0.so $L/libtrpo_mi355x.so"
