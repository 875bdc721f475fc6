tools/gpu_steps.sh 400 coop_tests.log 'python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_update.py tests/test_gpu_surrogate.py tests/test_gpu_ycache.py -x -q --timeout 120 --timeout-method thread' \
  120 coop_time.log 'python tools/update_only.py 2x64 50000 20 && python tools/update_only.py arm 50000 20 && python tools/cg_only.py 2x64 50000 20' \
  200 ab_rd.log 'SHAPES=2x64 ROUNDS=5 python tools/ab.py trpo-robot-control_amd/lib/libtrpo_mi355x.so trpo-robot-control_amd/lib/libtrpo_mi355x.so:TRPO_FUSE_REDUCE_DOTS=0'
