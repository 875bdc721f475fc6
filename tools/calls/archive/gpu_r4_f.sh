export TMPDIR=/tmp
tools/gpu_steps.sh \
  60 bisect_torch_threads.log 'python -u tools/diag/torch_first_bisect.py torch threads' \
  60 bisect_torch_group.log 'python -u tools/diag/torch_first_bisect.py torch group' \
  60 bisect_torch_fvp.log 'python -u tools/diag/torch_first_bisect.py torch fvp'
