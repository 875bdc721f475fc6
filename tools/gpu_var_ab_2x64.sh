#!/bin/bash
# interleaved A/B of lib/variants/*.so on the 2x64 policy (env NS: sample counts, default 4096 50000)
V=trpo-robot-control_amd/lib/variants
args=""; for v in "$@"; do args="$args $V/$v.so"; done
for n in ${NS:-4096 50000}; do
  SHAPES=2x64 N=$n ROUNDS=5 timeout -k 10 300 python tools/ab.py $args || exit 1
done
