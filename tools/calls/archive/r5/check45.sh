# round 5, call 45: atomic replica count (R) and grid size of the armDOF_0 CG on the final build
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
L=trpo-robot-control_amd/lib/libtrpo_mi355x.so
tools/gpu_steps.sh \
  300 r5/check45_ab_50k.log "SHAPES=arm N=50000 ROUNDS=11 python -u tools/ab.py $L $L:TRPO_REPLICAS=4 $L:TRPO_REPLICAS=8 $L:TRPO_FVP_BLOCKS=224 $L:TRPO_FVP_BLOCKS=196" \
  300 r5/check45_ab_6250.log "SHAPES=arm N=6250 ROUNDS=11 python -u tools/ab.py $L $L:TRPO_REPLICAS=4 $L:TRPO_REPLICAS=8"
