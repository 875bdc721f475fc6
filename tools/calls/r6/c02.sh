# round 6, call 2: knob cleanup + two tiles per trip in the cached-forward small-net kernels (TRPO_YC_NT=2):
# the GPU suite, smoke, an interleaved A/B against the one-tile build (lib/variants/nt1.so) at 50k / 500k / 4M,
# then the default bench line
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
tools/gpu_steps.sh \
  700 r6/c02_tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  120 r6/c02_smoke.log 'python -c "import __graft_entry__ as g; g.smoke()"' \
  300 r6/c02_ab.log 'for n in 50000 500000 4000000; do SHAPES=arm N=$n ROUNDS=5 python tools/ab.py trpo-robot-control_amd/lib/libtrpo_mi355x.so trpo-robot-control_amd/lib/variants/nt1.so || exit $?; done' \
  600 r6/c02_bench.log 'python bench.py > gpurun_out/r6/c02_bench.json'
