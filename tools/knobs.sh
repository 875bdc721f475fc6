#!/bin/bash
# CG(10) wall time for a few env-knob settings (armDOF_0, N from $1, default 50000)
n=${1:-50000}
for kv in "" "TRPO_REPLICAS=4" "TRPO_REPLICAS=6" "TRPO_REPLICAS=2" "TRPO_CG_REORTH=0" ""; do
  echo "== [$kv] N=$n"; env $kv timeout -k 5 60 python tools/cg_only.py arm $n 5 || exit $?
done
