tools/gpu_steps.sh 400 peer.log 'for i in 1 2 3; do python -u -m pytest tests/test_gpu_peer.py -x -q --timeout 120 --timeout-method thread || exit 1; done' \
  600 gputests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread'
