# round-4 final profiles: the 4M PMC traffic + SQ passes of the CG-iteration kernel, and a kernel
# trace of the 2x64 solve (per-iteration kernel durations)
export TMPDIR=/tmp
mkdir -p gpurun_out/cg2x64
bash tools/gpu_pmc_4m.sh && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cg2x64 -o run -- python3 tools/cg_only.py 2x64 50000 20 > gpurun_out/cg2x64/run.log 2>&1
