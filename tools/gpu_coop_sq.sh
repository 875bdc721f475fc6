export TMPDIR=/tmp
O=gpurun_out/coop_sq; mkdir -p $O
CG="python3 tools/cg_only.py 2x64 50000 5"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d $O/sq1 -o run -- $CG > $O/sq1.log 2>&1 && \
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_MISC --output-format csv -d $O/sq2 -o run -- $CG > $O/sq2.log 2>&1 && \
KERNEL="fvp_coop_kernel<float, 1, 4, 5, 3, 4>" python3 tools/pmc_summary.py $O/sq1 $O/sq2 > $O/sq_counters.txt 2>&1; cat $O/sq_counters.txt
