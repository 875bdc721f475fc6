#!/bin/bash
# interleaved A/B of lib/variants/*.so given as arguments (env NS: sample counts, default 50k 500k 4M)
V=trpo-robot-control_amd/lib/variants
args=""; for v in "$@"; do args="$args $V/$v.so"; done
for n in ${NS:-50000 500000 4000000}; do
  SHAPES=arm N=$n ROUNDS=5 timeout -k 10 240 python tools/ab.py $args || exit 1
done
