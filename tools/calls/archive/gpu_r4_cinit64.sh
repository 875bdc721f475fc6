# fp64 cooperative CG: the CG start inside the first FVP launch (default) vs cg_init (TRPO_COOP_CINIT=0):
# the GPU suite, then two bench runs (the C3 fp64 rows)
export TMPDIR=/tmp
mkdir -p gpurun_out/cinit64
tools/gpu_steps.sh \
  600 cinit64/tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  300 cinit64/bench_on.log 'python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-pmc' \
  300 cinit64/bench_off.log 'TRPO_COOP_CINIT=0 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-pmc' \
  300 cinit64/bench_on2.log 'python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-pmc'
