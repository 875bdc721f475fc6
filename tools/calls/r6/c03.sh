# round 6, call 3: the 2x64 CG step fused into the slab-reduce + dots launch (TRPO_COOP_AXF, default on):
# the cooperative / CG / update GPU tests, then the whole suite, an interleaved A/B (AXF on vs off) for 2x64
# at 50k and 4 096, and the C3 kernel trace
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
L=trpo-robot-control_amd/lib/libtrpo_mi355x.so
tools/gpu_steps.sh \
  300 r6/c03_coop_tests.log 'python -u -m pytest tests/test_gpu_coop_step.py tests/test_gpu_parity.py tests/test_gpu_update.py -m gpu -x -q --timeout 120 --timeout-method thread' \
  700 r6/c03_tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  300 r6/c03_ab.log "for n in 50000 4096; do SHAPES=2x64 N=\$n ROUNDS=7 timeout -k 5 100 python tools/ab.py $L $L:TRPO_COOP_AXF=0 || exit \$?; done" \
  200 r6/c03_trace.log 'rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6/c03_p2x64 -o run -- python3 tools/cg_only.py 2x64 50000 20'
