# round 5, call 46: 4-rank rehearsal of the N > 1 bench on one GPU with the final build (default flags)
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
tools/gpu_steps.sh 600 r5/check46_bench4.log 'TRPO_BENCH_DEVICE=0 python -u bench.py --gpus 4 --steps 20 --warmup 5'
