export TMPDIR=/tmp
tools/gpu_steps.sh \
  60 bisect_torch_none.log 'python -u tools/diag/torch_first_bisect.py torch none' \
  60 bisect_torch_create.log 'python -u tools/diag/torch_first_bisect.py torch create' \
  60 bisect_torch_handle.log 'python -u tools/diag/torch_first_bisect.py torch handle' \
  60 bisect_torch_attach.log 'python -u tools/diag/torch_first_bisect.py torch attach' \
  60 bisect_torch_update.log 'python -u tools/diag/torch_first_bisect.py torch update' \
  60 bisect_notorch_update.log 'python -u tools/diag/torch_first_bisect.py notorch update' \
  600 stall_hist3.log 'python -u tools/diag/stall_hist.py' \
  600 tests.log 'TRPO_TIMING_OUT=gpurun_out/r04_lbfgs_fit_timing.json python -u -m pytest tests -m gpu -v -s --timeout 120 --timeout-method thread'
