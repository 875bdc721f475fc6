# A/B of library variants (argument list) at N = 50k and 6 250, after the parity tests
tools/gpu_steps.sh 300 ab_tests.log 'python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ycache.py tests/test_gpu_properties.py -x -q --timeout 120 --timeout-method thread'   300 ab.log "SHAPES=arm ROUNDS=7 python tools/ab.py $* && SHAPES=arm N=6250 ROUNDS=7 python tools/ab.py $*"
