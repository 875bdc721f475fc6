#!/bin/bash
# effective clock of the CG-iteration kernel per library variant (args: lib/variants names), N=${N:-4000000}
export TMPDIR=/tmp
O=gpurun_out/clk; mkdir -p "$O"
for v in "$@"; do
  TRPO_LIB=trpo-robot-control_amd/lib/variants/$v.so timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace \
    --output-format csv -d "$O/$v" -o run -- python3 tools/cg_only.py arm ${N:-4000000} 2 > "$O/$v.log" 2>&1 || exit 1
  python3 tools/clock_summary.py "$O/$v" || exit 1
done
