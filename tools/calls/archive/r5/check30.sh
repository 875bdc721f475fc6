# round 5, call 30: cached-forward tile loop on a ring of input slots (no per-trip copies), depth 1 / 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
L=trpo-robot-control_amd/lib
tools/gpu_steps.sh \
  300 r5/check30_tests.log 'python -u -m pytest tests/test_gpu_ycache.py tests/test_gpu_narrow_out.py tests/test_gpu_parity.py tests/test_gpu_large_n.py -x -q --timeout 120 --timeout-method thread' \
  300 r5/check30_ab_4m.log "SHAPES=arm N=4000000 ROUNDS=7 python -u tools/ab.py $L/variants/ring0.so $L/libtrpo_mi355x.so $L/variants/ring2.so" \
  300 r5/check30_ab_500k.log "SHAPES=arm N=500000 ROUNDS=9 python -u tools/ab.py $L/variants/ring0.so $L/libtrpo_mi355x.so $L/variants/ring2.so" \
  300 r5/check30_ab_50k.log "SHAPES=arm N=50000 ROUNDS=9 python -u tools/ab.py $L/variants/ring0.so $L/libtrpo_mi355x.so $L/variants/ring2.so"
