# round 5 final measurements: kernel trace of the bench, PMC traffic and SQ counters of the CG-iteration
# kernel at 50k (tools/profile_round.sh) and at 4M (tools/gpu_pmc_4m.sh), the 2x64 solve's kernel trace
# (tools/gpu_prof_2x64.sh), and the driver's own bench command
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
bash tools/profile_round.sh r05 && bash tools/gpu_pmc_4m.sh && bash tools/gpu_prof_2x64.sh && \
tools/gpu_steps.sh 300 r5/final_bench_driver.log 'python -u bench.py --steps 20 --warmup 5'
