# round 5: cause of the peer-path wrong results under torch's runtime.  Each probe is its
# own process (torch imported first, the peer exchange allowed under it), bounded by its own time limit.
export TMPDIR=/tmp TRPO_PEER_ANY_RUNTIME=1
mkdir -p gpurun_out/r5_peer
P=tools/diag/torch_first_bisect.py
tools/gpu_steps.sh \
  120 r5_peer/close_alloc.log "TRPO_DEBUG_ALLOC=1 python -u $P torch fvp" \
  120 r5_peer/keep.log "python -u $P torch fvp keep" \
  120 r5_peer/keepwin.log "TRPO_PEER_KEEP_WINDOW=1 python -u $P torch fvp" \
  120 r5_peer/granule.log "TRPO_PEER_PROTO=2 python -u $P torch fvp" \
  120 r5_peer/nofence.log "TRPO_PEER_FENCE=0 python -u $P torch fvp" \
  120 r5_peer/notorch_alloc.log "TRPO_DEBUG_ALLOC=1 python -u $P notorch fvp"
