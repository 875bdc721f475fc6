#!/bin/bash
# narrow output layer: GPU tests, then interleaved A/B of the twins and the 16x16x4 output layer
L=trpo-robot-control_amd/lib/libtrpo_mi355x.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/no_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/no_tests.log
for n in 50000; do
  SHAPES=arm N=$n ROUNDS=5 timeout -k 10 240 python tools/ab.py $L:TRPO_NO_VALU_MIN_TILES=1000000 $L:TRPO_NO_VALU_MIN_TILES=0 $L:TRPO_NARROW_OUT=0 || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace2x64 -o run -- python3 tools/cg_only.py 2x64 50000 20 > gpurun_out/trace2x64.log 2>&1
echo "trace rc=$?"
