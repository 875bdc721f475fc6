# round 5, call 5: the segment-restructured cooperative kernel (no rotation) against the pre-restructure
# build (bits, time) and the GPU suite; the peer-path fix (uncached windows pooled, never freed) under
# torch's runtime: the round-4 reproduction, the granule / flag / update probes, and the same with the
# window freed again (TRPO_PEER_FREE_WINDOW) and the runtime's kernel-argument placement switched
export TMPDIR=/tmp
mkdir -p gpurun_out/r5 gpurun_out/r5_peer
L=trpo-robot-control_amd/lib
P="TRPO_PEER_ANY_RUNTIME=1 python -u tools/diag/torch_first_bisect.py"
tools/gpu_steps.sh \
  600 r5/check5_tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  300 r5/check5_ab_pre.log "SHAPES=2x64,arm ROUNDS=7 python -u tools/ab.py $L/variants/pre.so $L/libtrpo_mi355x.so $L/variants/coopprio.so" \
  300 r5/check5_ab_pre_4096.log "SHAPES=2x64 N=4096 ROUNDS=7 python -u tools/ab.py $L/variants/pre.so $L/libtrpo_mi355x.so $L/variants/coopprio.so" \
  240 r5_peer/repro_round4_pooled.log 'TRPO_PEER_ANY_RUNTIME=1 python -u tests/peer_torch_first.py any' \
  240 r5_peer/repro_round4_freed.log 'TRPO_PEER_FREE_WINDOW=1 TRPO_PEER_ANY_RUNTIME=1 python -u tests/peer_torch_first.py any' \
  120 r5_peer/granule_pooled.log "TRPO_PEER_PROTO=2 $P torch fvp" \
  120 r5_peer/flag_update_pooled.log "$P torch update" \
  120 r5_peer/granule_freed.log "TRPO_PEER_FREE_WINDOW=1 TRPO_PEER_PROTO=2 $P torch fvp" \
  120 r5_peer/flag_update_freed.log "TRPO_PEER_FREE_WINDOW=1 $P torch update" \
  120 r5_peer/granule_freed_kernarg0.log "HIP_FORCE_DEV_KERNARG=0 TRPO_PEER_FREE_WINDOW=1 TRPO_PEER_PROTO=2 $P torch fvp" \
  120 r5_peer/granule_freed_kernarg1.log "HIP_FORCE_DEV_KERNARG=1 TRPO_PEER_FREE_WINDOW=1 TRPO_PEER_PROTO=2 $P torch fvp" \
  120 r5_peer/granule_freed_notorch.log "TRPO_PEER_FREE_WINDOW=1 TRPO_PEER_PROTO=2 $P notorch fvp"
