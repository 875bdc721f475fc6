# round 5, call 2: the GPU suite again (restated stall-guard margin test), the suite with every device
# allocation poisoned (TRPO_DEBUG_POISON: reads of memory the library never wrote), the peer probe under
# poison, the s_setprio A/B and the coop phase stamps with and without it
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
L=trpo-robot-control_amd/lib
tools/gpu_steps.sh \
  600 r5/check2_tests.log 'TRPO_RITZ_LOG=gpurun_out/r5/ritz_margin.json python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  600 r5/check2_poison_tests.log 'TRPO_DEBUG_POISON=63 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider' \
  120 r5/check2_poison_peer.log 'TRPO_PEER_ANY_RUNTIME=1 TRPO_PEER_PROTO=2 TRPO_DEBUG_POISON=63 python -u tools/diag/torch_first_bisect.py torch fvp' \
  120 r5/check2_peer_granule_again.log 'TRPO_PEER_ANY_RUNTIME=1 TRPO_PEER_PROTO=2 python -u tools/diag/torch_first_bisect.py torch fvp' \
  120 r5/check2_peer_granule_notorch.log 'TRPO_PEER_ANY_RUNTIME=1 TRPO_PEER_PROTO=2 python -u tools/diag/torch_first_bisect.py notorch fvp' \
  300 r5/check2_ab_prio.log "ROUNDS=7 python -u tools/ab.py $L/libtrpo_mi355x.so $L/variants/prio.so" \
  300 r5/check2_ab_prio_4m.log "SHAPES=arm N=4000000 ROUNDS=5 python -u tools/ab.py $L/libtrpo_mi355x.so $L/variants/prio.so" \
  120 r5/check2_stamps.log 'python -u tools/stamps_coop.py 4096 50000' \
  120 r5/check2_stamps_prio.log "TRPO_LIB=$L/variants/prio_stamps.so python -u tools/stamps_coop.py 4096 50000"
