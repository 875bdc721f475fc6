#!/bin/bash
# waves per block of the small-net kernel at large N (variants lib/variants/w12.so, w16.so)
L=trpo-robot-control_amd/lib/libtrpo_mi355x.so
for n in 500000 4000000; do
  SHAPES=arm N=$n ROUNDS=5 timeout -k 10 240 python tools/ab.py $L trpo-robot-control_amd/lib/variants/w12.so trpo-robot-control_amd/lib/variants/w16.so || exit 1
done
