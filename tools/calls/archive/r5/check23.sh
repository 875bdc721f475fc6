# round 5, call 23: a 4-rank rehearsal of the N > 1 bench on ONE GPU with the default flags (RCCL refuses a
# second rank per device, so the headline falls back to the peer exchange -- the split granule form now);
# headline first, then the secondaries (RCCL again, the flag-form peer exchange, the sharded update) and
# the sweep, each behind its own agreement
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
tools/gpu_steps.sh 600 r5/check23_bench4.log 'TRPO_BENCH_DEVICE=0 python -u bench.py --gpus 4 --steps 20 --warmup 5'
