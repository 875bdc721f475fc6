# round 5, call 47: the tile loop's prefetch pin (sched_barrier after the loads) on the final build, on vs off
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
L=trpo-robot-control_amd/lib
A="$L/libtrpo_mi355x.so $L/variants/pin0.so"
tools/gpu_steps.sh \
  300 r5/check47_ab_4m.log "SHAPES=arm N=4000000 ROUNDS=7 python -u tools/ab.py $A" \
  300 r5/check47_ab_500k.log "SHAPES=arm N=500000 ROUNDS=9 python -u tools/ab.py $A" \
  300 r5/check47_ab_50k.log "SHAPES=arm,2x64 N=50000 ROUNDS=9 python -u tools/ab.py $A"
