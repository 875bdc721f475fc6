# round 6, call 21: HEAD as committed (docs and a renamed test since call 19) -- the whole GPU suite and smoke
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
tools/gpu_steps.sh \
  700 r6/c21_tests.log 'python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread' \
  120 r6/c21_smoke.log 'python -c "import __graft_entry__ as g; g.smoke()"'
