# small-net kernel: the transposed reads paired as ds_read2_b32 by an opaque per-slot LDS address
# (lib/variants/read2.so, built from /tmp/read2.patch) vs four ds_read_b32 (this build): interleaved A/B
# at 50k, 500k and 4M (x compared bit for bit), then the GPU suite on this build
export TMPDIR=/tmp
L=trpo-robot-control_amd/lib/libtrpo_mi355x.so
V=trpo-robot-control_amd/lib/variants
mkdir -p gpurun_out/read2
tools/gpu_steps.sh \
  300 read2/ab50k.log "SHAPES=arm ROUNDS=7 python -u tools/ab.py $L $V/read2.so" \
  300 read2/ab500k.log "SHAPES=arm ROUNDS=5 N=500000 python -u tools/ab.py $L $V/read2.so" \
  400 read2/ab4m.log "SHAPES=arm ROUNDS=5 N=4000000 python -u tools/ab.py $L $V/read2.so" \
  600 read2/tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread'
