bash tools/profile_round.sh r02 && TRPO_BENCH_DEVICE=0 tools/gpu_steps.sh 150 b2_rccl.log 'python bench.py --gpus 2 --steps 10 --warmup 2 --no-extra'
