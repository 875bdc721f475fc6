#!/bin/bash
# 2x64 CG A/B (fused reduce + dots, narrow output layer) and the bench-style single-context timing
L=trpo-robot-control_amd/lib/libtrpo_mi355x.so
for n in 4096 50000; do
  SHAPES=2x64 N=$n ROUNDS=5 timeout -k 10 240 python tools/ab.py $L $L:TRPO_NATSLAB=0 $L:TRPO_NARROW_OUT=0 $L:TRPO_NATSLAB=0,TRPO_NARROW_OUT=0 || exit 1
done
for e in "" "TRPO_NATSLAB=0 TRPO_NARROW_OUT=0"; do
  env $e timeout -k 10 120 python tools/cg_only.py 2x64 50000 20 || exit 1
done
