bash tools/calls/gpu_tests.sh > gpurun_out/tests_sgpr.log 2>&1 && NS="50000 500000" bash tools/gpu_var_ab.sh head final > gpurun_out/var_final.log 2>&1
