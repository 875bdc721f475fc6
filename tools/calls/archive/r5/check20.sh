# round 5, call 20 (VERDICT r04 #3 experiment): the small-net kernel without the register prefetch fits 126
# VGPRs, so 16 waves per block (4 per SIMD) run without spills; A/B at 4M and 50k against the default
# (8 waves, prefetch), 12 waves without prefetch, and 12 waves with it
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
L=trpo-robot-control_amd/lib
tools/gpu_steps.sh \
  400 r5/check20_ab_4m.log "SHAPES=arm N=4000000 ROUNDS=3 python -u tools/ab.py $L/libtrpo_mi355x.so $L/variants/nopf16.so $L/variants/nopf12.so $L/variants/w12.so" \
  300 r5/check20_ab_50k.log "SHAPES=arm ROUNDS=9 python -u tools/ab.py $L/libtrpo_mi355x.so $L/variants/nopf16.so $L/variants/nopf12.so $L/variants/w12.so" \
  300 r5/check20_ab_500k.log "SHAPES=arm N=500000 ROUNDS=5 python -u tools/ab.py $L/libtrpo_mi355x.so $L/variants/nopf16.so $L/variants/nopf12.so $L/variants/w12.so"
