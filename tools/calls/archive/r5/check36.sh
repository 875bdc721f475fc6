# round 5, call 36: waves per block of the small-net kernel again, after the scalar-fp32 build (8 / 12 / 16)
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
L=trpo-robot-control_amd/lib
V=$L/variants
A="$L/libtrpo_mi355x.so $V/w12.so $V/w16.so"
tools/gpu_steps.sh \
  300 r5/check36_ab_4m.log "SHAPES=arm N=4000000 ROUNDS=7 python -u tools/ab.py $A" \
  300 r5/check36_ab_500k.log "SHAPES=arm N=500000 ROUNDS=7 python -u tools/ab.py $A" \
  300 r5/check36_ab_50k.log "SHAPES=arm N=50000 ROUNDS=7 python -u tools/ab.py $A"
