# round 5, call 32: device code without packed fp32 VALU (v_pk_* beside MFMAs, MI355X_MICROARCH.md 'price of one filler')
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
L=trpo-robot-control_amd/lib
V=$L/variants
tools/gpu_steps.sh \
  300 r5/check32_ab_4m.log "SHAPES=arm N=4000000 ROUNDS=7 python -u tools/ab.py $L/libtrpo_mi355x.so $V/nopk.so" \
  300 r5/check32_ab_500k.log "SHAPES=arm N=500000 ROUNDS=9 python -u tools/ab.py $L/libtrpo_mi355x.so $V/nopk.so" \
  300 r5/check32_ab_50k.log "SHAPES=arm,2x64 N=50000 ROUNDS=9 python -u tools/ab.py $L/libtrpo_mi355x.so $V/nopk.so" \
  300 r5/check32_ab_4096.log "SHAPES=2x64 N=4096 ROUNDS=9 python -u tools/ab.py $L/libtrpo_mi355x.so $V/nopk.so"
