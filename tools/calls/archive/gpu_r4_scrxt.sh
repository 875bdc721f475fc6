# small-net kernel: tile transposes as one ds_write_b128 + transposed ds_read2_b32 (TRPO_SCR_XT=1, this
# build) vs the 4 ds_write_b32 + ds_read_b128 scratch (lib/variants/scr0.so): interleaved A/B at 50k,
# 500k and 4M, then the GPU suite
export TMPDIR=/tmp
L=trpo-robot-control_amd/lib/libtrpo_mi355x.so
V=trpo-robot-control_amd/lib/variants
mkdir -p gpurun_out/scrxt
tools/gpu_steps.sh \
  300 scrxt/ab50k.log "SHAPES=arm ROUNDS=7 python -u tools/ab.py $L $V/scr0.so" \
  300 scrxt/ab500k.log "SHAPES=arm ROUNDS=5 N=500000 python -u tools/ab.py $L $V/scr0.so" \
  400 scrxt/ab4m.log "SHAPES=arm ROUNDS=3 N=4000000 python -u tools/ab.py $L $V/scr0.so" \
  600 scrxt/tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread'
