#!/bin/bash
# forward-activation cache on/off per N (TRPO_YCACHE=0: every CG iteration recomputes the forward pass)
L=trpo-robot-control_amd/lib/libtrpo_mi355x.so
for n in ${NS:-50000 500000 1000000 2000000 4000000}; do
  SHAPES=arm N=$n ROUNDS=5 timeout -k 10 240 python tools/ab.py $L $L:TRPO_YCACHE=0 || exit 1
done
