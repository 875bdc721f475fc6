# round 5, call 34: scheduler options of the device compile (max-ilp strategy, latency-biased metric, MFMA VGPR form)
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
L=trpo-robot-control_amd/lib
V=$L/variants
A="$L/libtrpo_mi355x.so $V/maxilp.so $V/bias0.so $V/vgprform.so"
tools/gpu_steps.sh \
  300 r5/check34_ab_50k.log "SHAPES=arm,2x64 N=50000 ROUNDS=7 python -u tools/ab.py $A" \
  300 r5/check34_ab_4m.log "SHAPES=arm N=4000000 ROUNDS=5 python -u tools/ab.py $A" \
  300 r5/check34_ab_500k.log "SHAPES=arm N=500000 ROUNDS=7 python -u tools/ab.py $A" \
  300 r5/check34_ab_4096.log "SHAPES=2x64 N=4096 ROUNDS=7 python -u tools/ab.py $A"
