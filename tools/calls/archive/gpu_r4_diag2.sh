export TMPDIR=/tmp
tools/gpu_steps.sh \
  150 tfs_torch.log 'python -u tools/diag/torch_first_seq.py torch 3' \
  150 tfs_notorch.log 'python -u tools/diag/torch_first_seq.py notorch 2' \
  300 warm_ab.log 'python -u tools/warm_ab.py 3' \
  400 ab_splitk.log 'NS="50000 500000 4000000" bash tools/gpu_var_ab.sh base splitk'
