# round 6, call 6: A/B of the tile -> wave mapping beyond the first round (TRPO_TILE_SPREAD=1 spreads the
# later rounds over the blocks, 0 keeps them block-major) on the arm net at four sizes
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
V=trpo-robot-control_amd/lib/variants
tools/gpu_steps.sh \
  400 r6/c06_ab.log "for n in 50000 6250 500000 4000000; do SHAPES=arm N=\$n ROUNDS=7 timeout -k 5 100 python tools/ab.py $V/spread0.so $V/spread1.so || exit \$?; done"
