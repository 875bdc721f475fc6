# round-4 last measurement on the final build: the default bench line (traffic measured in the run) and
# a kernel trace of the 2x64 solve
export TMPDIR=/tmp
mkdir -p gpurun_out/last
tools/gpu_steps.sh \
  600 last/bench.log 'python -u bench.py' \
  200 last/trace2x64.log 'rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/last/cg2x64 -o run -- python3 tools/cg_only.py 2x64 50000 20'
