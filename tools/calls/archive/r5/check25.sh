# round 5, call 25: the baseline evaluate at N = 64 / 640 / 3000 / 12000 under a kernel trace
export TMPDIR=/tmp
mkdir -p gpurun_out/r5/bn
tools/gpu_steps.sh 180 r5/bn/bn.log "rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5/bn/tr -o run -- python3 tools/diag/baseline_n.py"
