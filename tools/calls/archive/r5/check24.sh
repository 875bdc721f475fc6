# round 5, call 24: kernel trace of the caller's liblbfgs baseline fit on the device evaluate (C5's larger part)
export TMPDIR=/tmp
mkdir -p gpurun_out/r5/fit
tools/gpu_steps.sh 180 r5/fit/fit.log "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/fit/tr -o run -- python3 tests/lbfgs_fit_child.py 5"
