# round 6, call 7: where a baseline evaluate's ~28 us go -- host wait forms (tools/micro/host_wait), the
# evaluate's host-visible time and the caller's liblbfgs fit, and the kernel trace of the evaluate loop
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
tools/gpu_steps.sh \
  120 r6/c07_host_wait.log 'tools/micro/host_wait' \
  240 r6/c07_eval.log 'python tools/baseline_eval_timing.py 3000' \
  200 r6/c07_eval_trace.log 'rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6/c07_trace -o run -- python3 tools/baseline_eval_timing.py 500'
