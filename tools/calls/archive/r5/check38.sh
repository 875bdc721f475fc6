# round 5, call 38: standalone FVP calls on group-major tiles up to one tile per CU (CG launches unchanged)
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
L=trpo-robot-control_amd/lib/libtrpo_mi355x.so
tools/gpu_steps.sh \
  600 r5/check38_tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  300 r5/check38_ab_4096.log "SHAPES=2x64 N=4096 ROUNDS=11 python -u tools/ab.py $L:TRPO_COOP_GMAJ=0 $L" \
  300 r5/check38_ab_2048.log "SHAPES=2x64 N=2048 ROUNDS=9 python -u tools/ab.py $L:TRPO_COOP_GMAJ=0 $L" \
  300 r5/check38_ab_3000.log "SHAPES=2x64 N=3000 ROUNDS=9 python -u tools/ab.py $L:TRPO_COOP_GMAJ=0 $L" \
  300 r5/check38_ab_50k.log "SHAPES=2x64,arm N=50000 ROUNDS=7 python -u tools/ab.py $L:TRPO_COOP_GMAJ=0 $L"
