# round 5, call 17: loads the compiler had sunk under conditions (cg_axpy's partial dots, cg_last's replica
# sums, the slab reduces' first round and the FVP epilogue's direction gather) issued with the first round:
# GPU suite, then A/B against the previous kernels (prev.so) -- armDOF_0 and 2x64 at 50k, 2x64 at 4096
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
L=trpo-robot-control_amd/lib
tools/gpu_steps.sh \
  600 r5/check17_tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  300 r5/check17_ab.log "SHAPES=arm,2x64 ROUNDS=9 python -u tools/ab.py $L/variants/prev.so $L/libtrpo_mi355x.so" \
  300 r5/check17_ab_4096.log "SHAPES=2x64 N=4096 ROUNDS=9 python -u tools/ab.py $L/variants/prev.so $L/libtrpo_mi355x.so"
