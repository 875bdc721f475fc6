# round 5, call 41: cg_last_kernel's loads pinned before its done test (two memory round trips instead of three)
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
L=trpo-robot-control_amd/lib
tools/gpu_steps.sh \
  300 r5/check41_tests.log 'python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_coop_step.py tests/test_gpu_narrow_out.py tests/test_gpu_ycache.py tests/test_gpu_update.py tests/test_gpu_stall_guard.py -x -q --timeout 120 --timeout-method thread' \
  300 r5/check41_ab_50k.log "SHAPES=arm N=50000 ROUNDS=15 python -u tools/ab.py $L/variants/prevlast.so $L/libtrpo_mi355x.so" \
  300 r5/check41_ab_6250.log "SHAPES=arm N=6250 ROUNDS=15 python -u tools/ab.py $L/variants/prevlast.so $L/libtrpo_mi355x.so"
