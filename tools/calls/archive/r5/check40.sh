# round 5, call 40: the final build -- smoke(), the driver's bench command
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
tools/gpu_steps.sh \
  300 r5/check40_smoke.log 'python -u -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")"' \
  400 r5/check40_bench.log 'python -u bench.py --steps 20 --warmup 5'
