#!/bin/bash
# PMC traffic passes (FETCH_SIZE, WRITE_SIZE) of the CG-iteration kernel at N = 4M (throughput regime)
O=gpurun_out/pmc4m
mkdir -p "$O"
export TMPDIR=/tmp
CG="python3 tools/cg_only.py arm 4000000 2"
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch" -o run -- $CG > "$O/fetch.log" 2>&1 && \
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write" -o run -- $CG > "$O/write.log" 2>&1 && \
F=$(find "$O/fetch" -name '*counter_collection.csv' | head -1) && W=$(find "$O/write" -name '*counter_collection.csv' | head -1) && \
KERNEL="fvp_mlp3_kernel<1, 1, 1, 1, 5, 3" LABEL="CG-iteration kernel (MODE 3), N = 4M" WORKLOAD="armDOF_0 N=4000000" \
    python3 tools/pmc_traffic.py "$F" "$W" "$O/cgiter_traffic_4m.json"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d "$O/sq1" -o run -- $CG > "$O/sq1.log" 2>&1 && \
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU \
    SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_MISC --output-format csv -d "$O/sq2" -o run -- $CG > "$O/sq2.log" 2>&1 && \
KERNEL="fvp_mlp3_kernel<1, 1, 1, 1, 5, 3" python3 tools/pmc_summary.py "$O/sq1" "$O/sq2" > "$O/sq_counters_4m.txt" 2>&1
