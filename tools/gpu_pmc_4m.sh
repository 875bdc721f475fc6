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
