# round 6, call 8: by-value 4.5 KB kernel argument on gfx950 (tools/micro/kernarg_big), the evaluate's
# host-visible time + liblbfgs fit, and the kernel trace of the evaluate loop
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
tools/gpu_steps.sh \
  120 r6/c08_kernarg.log 'tools/micro/kernarg_big' \
  240 r6/c08_eval.log 'python tools/baseline_eval_timing.py 3000' \
  200 r6/c08_eval_trace.log 'rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6/c08_trace -o run -- python3 tools/baseline_eval_timing.py 500'
