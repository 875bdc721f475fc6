export TMPDIR=/tmp
tools/gpu_steps.sh \
  600 tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  300 launch_form_ab2.log 'python -u tools/launch_form_ab.py' \
  300 bench2ranks.log 'TRPO_BENCH_DEVICE=0 python -u bench.py --gpus 2 --steps 50 --warmup 5' \
  300 bench2ranks_nofence.log 'TRPO_PEER_FENCE=0 TRPO_BENCH_DEVICE=0 python -u bench.py --gpus 2 --steps 50 --warmup 5 --no-extra --no-cpu-baseline'
