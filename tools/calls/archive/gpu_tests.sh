#!/bin/bash
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/tests.log; exit $rc
