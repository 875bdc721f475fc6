# round 5 final measurements (second pass, the final kernels): kernel trace of the bench, PMC traffic and SQ
# counters of the CG-iteration kernel at 50k and 4M, the 2x64 solve's kernel trace, the driver's own bench
# command, and the one-GPU peer exchange floor of the default form
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
bash tools/profile_round.sh r05b && bash tools/gpu_pmc_4m.sh && bash tools/gpu_prof_2x64.sh && \
tools/gpu_steps.sh 300 r5/final2_bench_driver.log 'python -u bench.py --steps 20 --warmup 5' \
  240 r5/final2_pf.log "rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5/final2_pf -o run -- python3 tools/peer_floor.py" \
  60 r5/final2_pf_stats.log "python3 tools/peer_floor_stats.py proto4 gpurun_out/r5/final2_pf"
