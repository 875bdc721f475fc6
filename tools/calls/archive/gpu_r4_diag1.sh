export TMPDIR=/tmp
tools/gpu_steps.sh \
  120 tf_notorch.log 'python -u tools/diag/torch_first_fvp.py notorch' \
  120 tf_torch.log 'python -u tools/diag/torch_first_fvp.py torch' \
  900 stall_hist.log 'python -u tools/diag/stall_hist.py'
