# round 5, call 33: no packed fp32 VALU in the default build -- GPU suite, ring A/B, default bench line
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
L=trpo-robot-control_amd/lib
V=$L/variants
tools/gpu_steps.sh \
  600 r5/check33_tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  300 r5/check33_ab_4m.log "SHAPES=arm N=4000000 ROUNDS=7 python -u tools/ab.py $V/ring0.so $L/libtrpo_mi355x.so" \
  300 r5/check33_ab_500k.log "SHAPES=arm N=500000 ROUNDS=9 python -u tools/ab.py $V/ring0.so $L/libtrpo_mi355x.so" \
  300 r5/check33_ab_50k.log "SHAPES=arm N=50000 ROUNDS=9 python -u tools/ab.py $V/ring0.so $L/libtrpo_mi355x.so" \
  400 r5/check33_bench.log 'python -u bench.py --steps 20 --warmup 5'
