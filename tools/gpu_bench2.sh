# two bench ranks on ONE GPU (TRPO_BENCH_DEVICE=0): the multi-rank bench path with the peer exchange
export TRPO_BENCH_DEVICE=0
tools/gpu_steps.sh 180 b2_peer.log 'python bench.py --gpus 2 --comm peer --steps 20 --warmup 3 --no-extra' \
                   180 b2_peer_extra.log 'python bench.py --gpus 2 --comm peer --steps 20 --warmup 3'
