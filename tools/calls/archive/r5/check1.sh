# round 5, first check of the new build: GPU suite (incl. the stall-guard margin table), smoke, the
# driver's bench command, then the peer-path probes (tools/calls/r5/peer_probe.sh)
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
tools/gpu_steps.sh \
  900 r5/check1_tests.log 'TRPO_RITZ_LOG=gpurun_out/r5/ritz_margin.json python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  200 r5/check1_smoke.log 'python -u -c "import __graft_entry__ as g; g.smoke()"' \
  400 r5/check1_bench.log 'python -u bench.py --steps 20 --warmup 5' && bash tools/calls/r5/peer_probe.sh
tools/gpu_steps.sh 120 r5/stamps_coop.log 'python -u tools/stamps_coop.py 4096 50000'
