# round 5 final measurements (third pass, after the baseline-evaluate kernels): baseline tests, the bench's
# kernel trace / PMC traffic / SQ counters (50k), the 4M counters, the 2x64 trace, the driver's bench command
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
tools/gpu_steps.sh 300 r5/final3_baseline_tests.log "python -u -m pytest tests/test_gpu_baseline.py tests/test_lbfgs_caller.py -x -q --timeout 180 --timeout-method thread" && \
bash tools/profile_round.sh r05c && bash tools/gpu_pmc_4m.sh && bash tools/gpu_prof_2x64.sh && \
tools/gpu_steps.sh 300 r5/final3_bench_driver.log 'python -u bench.py --steps 20 --warmup 5'
