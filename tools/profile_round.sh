#!/bin/bash
# One GPU call that refreshes the round's measurements of the kernel in the timed region (the fused
# CG-iteration kernel fvp_mlp3_kernel<...,3,QB>, MODE 3) and the bench line.
#   tools/profile_round.sh rNN          (run on the GPU box from the repo root)
# Steps (each under its own time limit; the first failure ends the script):
#   1. rocprofv3 kernel trace of bench.py (timed CG solves)            -> trace_bench/*kernel_stats.csv
#   2. two separate PMC passes (FETCH_SIZE, WRITE_SIZE) of CG solves    -> cgiter_traffic.json
#   3. two SQ counter passes of the same CG solves                      -> sq_counters.txt
#   4. bench.py (headline + extras + CPU baseline) reading that traffic -> bench.json
# Outputs under gpurun_out/prof_rNN/; copy the summaries into profiles/ afterwards.
R=${1:?round tag, e.g. r02}
O=gpurun_out/prof_$R
mkdir -p "$O"
export TMPDIR=/tmp
step() {
    local t=$1 name=$2
    shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "[profile] $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -20 "$O/$name.log"; exit $rc; fi
}
CG="python3 tools/cg_only.py arm 50000 5"
step 300 trace_bench rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_bench" -o run -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra
step 120 pmc_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o run -- $CG
step 120 pmc_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o run -- $CG
F=$(find "$O/pmc_fetch" -name '*counter_collection.csv' | head -1)
W=$(find "$O/pmc_write" -name '*counter_collection.csv' | head -1)
KERNEL="fvp_mlp3_kernel<1, 1, 1, 1, 5, 3" LABEL="CG-iteration kernel (MODE 3, all QB variants)" \
    python3 tools/pmc_traffic.py "$F" "$W" "$O/cgiter_traffic.json" > "$O/traffic.log" 2>&1
echo "[profile] traffic rc=$?"
step 120 sq1 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d "$O/sq1" -o run -- $CG
step 120 sq2 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU \
    SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_MISC --output-format csv -d "$O/sq2" -o run -- $CG
KERNEL="fvp_mlp3_kernel<1, 1, 1, 1, 5, 3" python3 tools/pmc_summary.py "$O/sq1" "$O/sq2" > "$O/sq_counters.txt" 2>&1
TRPO_TRAFFIC_JSON="$O/cgiter_traffic.json" step 600 bench python3 bench.py
grep '^{' "$O/bench.log" | tail -1 > "$O/bench.json"
find "$O" -name '*kernel_stats.csv' -o -name '*.json' -o -name '*.txt' | sort
