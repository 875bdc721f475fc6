export TMPDIR=/tmp
tools/gpu_steps.sh \
  60 uc_torch_uc.log 'python -u tools/diag/uc_recycle.py torch uc' \
  60 uc_torch_plain.log 'python -u tools/diag/uc_recycle.py torch plain' \
  60 uc_notorch_uc.log 'python -u tools/diag/uc_recycle.py notorch uc'
