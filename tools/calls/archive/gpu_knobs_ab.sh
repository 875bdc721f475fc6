#!/bin/bash
# 50k knob re-tune on the narrow-output kernel: atomic replicas, grid size
L=trpo-robot-control_amd/lib/libtrpo_mi355x.so
SHAPES=arm N=50000 ROUNDS=7 timeout -k 10 300 python tools/ab.py $L $L:TRPO_REPLICAS=4 $L:TRPO_REPLICAS=5 $L:TRPO_REPLICAS=8 $L:TRPO_FVP_BLOCKS=240 $L:TRPO_FVP_BLOCKS=224
