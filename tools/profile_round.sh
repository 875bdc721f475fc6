#!/bin/bash
# One GPU call that refreshes every measurement the round's profiles/ carry.
#   tools/profile_round.sh rNN          (run on the GPU box from the repo root)
# Steps (each under its own time limit; the first failure ends the script):
#   1. rocprofv3 kernel trace of bench  -> bench_kernel_stats.csv (every kernel of the timed CG solves)
#   2. rocprofv3 kernel trace of the FVP kernel alone (tools/kernel_only.py) -> fvp_kernel_stats.csv
#   3. two separate PMC passes (FETCH_SIZE, WRITE_SIZE) of the same launches -> traffic json
#   4. bench.py --extra with that traffic -> bench.json (headline line + the C2/C3/fp64/update/baseline extras)
# Outputs under gpurun_out/prof_rNN/; copy the summaries into profiles/ afterwards.
R=${1:?round tag, e.g. r01}
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
step 300 trace_bench rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_bench" -o run -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline
step 300 trace_fvp rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_fvp" -o run -- \
    python3 tools/kernel_only.py
step 300 pmc_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o run -- \
    python3 tools/kernel_only.py
step 300 pmc_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o run -- \
    python3 tools/kernel_only.py
F=$(find "$O/pmc_fetch" -name '*counter_collection.csv' | head -1)
W=$(find "$O/pmc_write" -name '*counter_collection.csv' | head -1)
python3 tools/pmc_traffic.py "$F" "$W" "$O/fvp_traffic.json" > "$O/traffic.log" 2>&1
echo "[profile] traffic rc=$?"
# the bench line last, reading the traffic measured just above
TRPO_TRAFFIC_JSON="$O/fvp_traffic.json" step 600 bench python3 bench.py --extra
grep '^{' "$O/bench.log" | tail -1 > "$O/bench.json"
find "$O" -name '*kernel_stats.csv' -o -name '*.json' | sort
