tools/gpu_steps.sh 300 surr_tests.log 'python -u -m pytest tests/test_gpu_surrogate.py tests/test_gpu_update.py -x -q --timeout 120 --timeout-method thread' \
  120 surr_time.log 'python tools/update_only.py 2x64 50000 20 && TRPO_SURR_GENERIC=1 python tools/update_only.py 2x64 50000 20 && python tools/update_only.py arm 50000 20' \
  180 surr_trace.log 'rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/surr_trace -o run -- python3 tools/update_only.py 2x64 50000 10'
