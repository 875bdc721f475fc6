#!/bin/bash
# round-3 check: GPU tests, the 2x64 A/Bs (fused reduce + dots, narrow output layer), the spill-variant diag
L=trpo-robot-control_amd/lib/libtrpo_mi355x.so
bash tools/calls/gpu_tests.sh || exit 1
for n in 4096 50000; do
  SHAPES=2x64 N=$n ROUNDS=5 timeout -k 10 240 python tools/ab.py $L $L:TRPO_NATSLAB=0 $L:TRPO_NARROW_OUT=0 $L:TRPO_NATSLAB=0,TRPO_NARROW_OUT=0 || exit 1
done
if [ -f trpo-robot-control_amd/lib/variants/yc1441.so ]; then
  timeout -k 10 200 python tools/diag/yc1441.py 50000 > gpurun_out/yc1441_50k.log 2>&1 || exit 1
  timeout -k 10 200 python tools/diag/yc1441.py 333 > gpurun_out/yc1441_333.log 2>&1 || exit 1
fi
