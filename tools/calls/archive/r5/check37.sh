# round 5, call 37: group-major cooperative tiles at N = 4 096 re-measured on the scalar-fp32 build
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
L=trpo-robot-control_amd/lib
tools/gpu_steps.sh \
  300 r5/check37_ab_4096.log "SHAPES=2x64 N=4096 ROUNDS=11 python -u tools/ab.py $L/libtrpo_mi355x.so $L/libtrpo_mi355x.so:TRPO_COOP_GMAJ=1" \
  300 r5/check37_ab_6144.log "SHAPES=2x64 N=6144 ROUNDS=9 python -u tools/ab.py $L/libtrpo_mi355x.so $L/libtrpo_mi355x.so:TRPO_COOP_GMAJ=1"
