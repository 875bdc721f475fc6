# round 6, call 4: the round's profiles on the final kernels -- rocprofv3 kernel trace of bench.py, PMC
# traffic + SQ counters of the CG-iteration kernel at 50k (tools/profile_round.sh) and at 4M
# (tools/gpu_pmc_4m.sh), the 2x64 CG trace, and the driver's own bench command
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
bash tools/profile_round.sh r06 > gpurun_out/r6/c04_profile_round.log 2>&1 && \
bash tools/gpu_pmc_4m.sh > gpurun_out/r6/c04_pmc4m.log 2>&1 && \
bash tools/gpu_prof_2x64.sh > gpurun_out/r6/c04_p2x64.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r6/c04_bench_steps20_warmup5.json 2> gpurun_out/r6/c04_bench_steps20.err
echo "c04 rc=$?"
