#!/bin/bash
# SQ counter passes on the FVP kernel alone (tools/kernel_only.py), one rocprofv3 run per pass.
#   tools/pmc_sq.sh OUTDIR N [N ...]
O=${1:?outdir}; shift
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 5 60 rocprofv3 -L > "$O/counters.txt" 2>&1
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_MISC"
for n in "$@"; do
  i=0
  for p in "$P1" "$P2"; do
    i=$((i+1))
    N=$n REPS=20 timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d "$O/n${n}_p$i" -o run -- \
        python3 tools/kernel_only.py > "$O/n${n}_p$i.log" 2>&1
    rc=$?
    echo "[pmc] n=$n pass=$i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$O/n${n}_p$i.log"; exit $rc; fi
  done
done
