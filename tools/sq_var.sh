#!/bin/bash
# SQ LDS pass for a variant lib: /tmp-free version lives in tools/ when kept
V=$1; name=$2
export TMPDIR=/tmp
TRPO_LIB=$V timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES --output-format csv -d gpurun_out/sqv_$name -o run -- python3 tools/cg_only.py arm 50000 5 > gpurun_out/sqv_$name.log 2>&1 || exit $?
KERNEL="fvp_mlp3_kernel<1, 1, 1, 1, 5, 3" python3 tools/pmc_summary.py gpurun_out/sqv_$name
