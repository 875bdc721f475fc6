# round 5, call 3: the rotated cooperative schedule (TRPO_COOP_ROT, default on) -- GPU suite, A/B against
# the unrotated build, phase stamps; the peer-path anomaly under torch's runtime with the runtime's own
# serialisation knobs (AMD_SERIALIZE_KERNEL, one hardware queue) and without the forward cache
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
L=trpo-robot-control_amd/lib
P="TRPO_PEER_ANY_RUNTIME=1 TRPO_PEER_PROTO=2 python -u tools/diag/torch_first_bisect.py"
tools/gpu_steps.sh \
  600 r5/check3_tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  300 r5/check3_ab_rot.log "SHAPES=2x64 ROUNDS=7 python -u tools/ab.py $L/variants/rot0.so $L/libtrpo_mi355x.so" \
  300 r5/check3_ab_rot_4096.log "SHAPES=2x64 N=4096 ROUNDS=7 python -u tools/ab.py $L/variants/rot0.so $L/libtrpo_mi355x.so" \
  120 r5/check3_stamps_rot.log 'python -u tools/stamps_coop.py 4096 50000' \
  120 r5/check3_peer_base.log "$P torch fvp" \
  120 r5/check3_peer_serialize.log "AMD_SERIALIZE_KERNEL=3 $P torch fvp" \
  120 r5/check3_peer_1queue.log "GPU_MAX_HW_QUEUES=1 $P torch fvp" \
  120 r5/check3_peer_noyc.log "TRPO_YCACHE=0 $P torch fvp" \
  120 r5/check3_peer_update.log "$P torch update"
