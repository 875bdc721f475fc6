tools/gpu_steps.sh 300 peer.log 'python -u -m pytest tests/test_gpu_peer.py tests/test_gpu_shard.py -x -v --timeout 120 --timeout-method thread'
