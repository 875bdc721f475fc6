# round 5, call 31: 4M bound analysis -- ring depths, input-stream-only and compute-only builds, clock counters
export TMPDIR=/tmp
mkdir -p gpurun_out/r5/clk
L=trpo-robot-control_amd/lib
V=$L/variants
CG="python3 tools/cg_only.py arm 4000000 2"
tools/gpu_steps.sh \
  300 r5/check31_ab_4m.log "SHAPES=arm N=4000000 ROUNDS=7 python -u tools/ab.py $V/ring0.so $L/libtrpo_mi355x.so $V/ring2.so $V/nocomp.so $V/noload.so" \
  300 r5/check31_ab_500k.log "SHAPES=arm N=500000 ROUNDS=9 python -u tools/ab.py $V/ring0.so $L/libtrpo_mi355x.so $V/ring2.so" \
  120 r5/clk/lib.log "timeout -s KILL 100 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVE_CYCLES --output-format csv -d gpurun_out/r5/clk/lib -o run -- $CG" \
  120 r5/clk/noload.log "TRPO_LIB=$V/noload.so timeout -s KILL 100 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVE_CYCLES --output-format csv -d gpurun_out/r5/clk/noload -o run -- $CG" \
  120 r5/clk/nocomp.log "TRPO_LIB=$V/nocomp.so timeout -s KILL 100 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/r5/clk/nocomp -o run -- $CG" \
  60 r5/clk/summary.txt "KERNEL='fvp_mlp3_kernel<1, 1, 1, 1, 5, 3' python3 tools/pmc_summary.py gpurun_out/r5/clk/lib gpurun_out/r5/clk/noload gpurun_out/r5/clk/nocomp"
