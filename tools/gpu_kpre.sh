tools/gpu_steps.sh 400 kpre_tests.log 'python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ycache.py tests/test_gpu_peer.py tests/test_gpu_comm.py -x -q --timeout 120 --timeout-method thread' \
  300 ab_kpre.log 'SHAPES=arm ROUNDS=7 python tools/ab.py trpo-robot-control_amd/lib/libtrpo_mi355x.so trpo-robot-control_amd/lib/variants/nokpre.so && SHAPES=arm N=6250 ROUNDS=7 python tools/ab.py trpo-robot-control_amd/lib/libtrpo_mi355x.so trpo-robot-control_amd/lib/variants/nokpre.so' \
  120 stamps.log 'REPL=6 WIDE=0 NS=50000,6250 python tools/stamps_cg.py'
