#!/bin/bash
# 2x64 CG(10) at N=50k and 4096: distributed CG step (default) vs the fused cooperative step; fp32 and fp64
for n in 50000 4096; do
  for kv in "TRPO_COOP_DIST=1" "TRPO_COOP_DIST=0"; do
    echo "== [$kv] N=$n"; env $kv timeout -k 5 60 python tools/cg_only.py 2x64 $n 5 || exit $?
  done
done
