# one-tile contractions' transposed reads as explicit ds_read2_b32 (lib/variants/asm2.so, TRPO_SCR_XT=2)
# vs the compiler's ds_read_b32 form (this build): interleaved A/B at 50k, 500k and 4M
export TMPDIR=/tmp
L=trpo-robot-control_amd/lib/libtrpo_mi355x.so
V=trpo-robot-control_amd/lib/variants
mkdir -p gpurun_out/asm2
tools/gpu_steps.sh \
  300 asm2/ab50k.log "SHAPES=arm ROUNDS=7 python -u tools/ab.py $L $V/asm2.so" \
  300 asm2/ab500k.log "SHAPES=arm ROUNDS=5 N=500000 python -u tools/ab.py $L $V/asm2.so" \
  400 asm2/ab4m.log "SHAPES=arm ROUNDS=5 N=4000000 python -u tools/ab.py $L $V/asm2.so"
