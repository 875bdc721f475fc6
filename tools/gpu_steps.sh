#!/bin/bash
# Run GPU steps in order; each under its own time limit.  A step that ends with anything but
# success or ordinary test failures (rc 0/1) -- a fault, abort, segfault or time limit -- stops
# the sequence.  Usage: tools/gpu_steps.sh SECONDS LOG 'cmd' [SECONDS LOG 'cmd' ...]
mkdir -p gpurun_out
while [ $# -ge 3 ]; do
    t=$1; log=$2; cmd=$3; shift 3
    timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/$log" 2>&1
    rc=$?
    echo "[step] $log rc=$rc"
    tail -3 "gpurun_out/$log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[step] stopping after rc=$rc"; exit $rc; fi
done
