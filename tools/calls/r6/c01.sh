# round 6, call 1: the GPU suite on the round-6 fixes (vpack after graph replay, peer error records,
# window-pool policy), smoke, and the default bench line (roofline.mfma_busy_frac measured in-run)
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
tools/gpu_steps.sh \
  700 r6/c01_tests.log 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  120 r6/c01_smoke.log 'python -c "import __graft_entry__ as g; g.smoke()"' \
  600 r6/c01_bench.log 'python bench.py > gpurun_out/r6/c01_bench.json'
