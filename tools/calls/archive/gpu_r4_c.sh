# round 4: host-group copies as hipMemcpyAsync (is the stale-copy rule still needed?),
# the 8-process peer rehearsal under a kernel trace (the exchange kernel's cost), the stall-guard
# statistic per golden / draw, and the fp32 stall-guard tests
export TMPDIR=/tmp
tools/gpu_steps.sh \
  200 shard_race_memcpy.log 'TRPO_LIB=trpo-robot-control_amd/lib/variants/hgmemcpy.so python -u tools/diag/shard_race.py group 10' \
  200 shard_race_kernels.log 'python -u tools/diag/shard_race.py group 10' \
  300 peer8_trace.log 'rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/peer8 -o run -- python3 -m pytest tests/test_gpu_peer.py -k "ipc_processes and 8" -x -q' \
  600 stall_hist2.log 'python -u tools/diag/stall_hist.py' \
  300 rand_shapes.log 'TRPO_TIMING_OUT=gpurun_out/r04_lbfgs_fit_timing.json python -u -m pytest tests/test_gpu_random_shapes.py tests/test_lbfgs_caller.py -x -q -s --timeout 120 --timeout-method thread'
tools/gpu_steps.sh \
  150 poison_notorch.log 'python -u tools/diag/poison_fvp.py notorch' \
  150 poison_torch.log 'python -u tools/diag/poison_fvp.py torch'
