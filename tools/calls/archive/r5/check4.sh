# round 5, call 4: the rotated cooperative schedule with a wave-uniform group index (GPU suite, A/B, stamps);
# the peer-path anomaly (granule form, torch's runtime): window leaked / contexts kept / allocation dump
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
L=trpo-robot-control_amd/lib
P="TRPO_PEER_ANY_RUNTIME=1 TRPO_PEER_PROTO=2 python -u tools/diag/torch_first_bisect.py"
tools/gpu_steps.sh \
  600 r5/check4_tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  300 r5/check4_ab_rot.log "SHAPES=2x64 ROUNDS=7 python -u tools/ab.py $L/variants/rot0.so $L/libtrpo_mi355x.so $L/variants/rotprio.so" \
  300 r5/check4_ab_rot_4096.log "SHAPES=2x64 N=4096 ROUNDS=7 python -u tools/ab.py $L/variants/rot0.so $L/libtrpo_mi355x.so $L/variants/rotprio.so" \
  120 r5/check4_stamps_rot.log 'python -u tools/stamps_coop.py 4096 50000' \
  120 r5/check4_peer_keepwin.log "TRPO_PEER_KEEP_WINDOW=1 $P torch fvp" \
  120 r5/check4_peer_keep.log "$P torch fvp keep" \
  120 r5/check4_peer_alloc.log "TRPO_DEBUG_ALLOC=1 $P torch fvp"
