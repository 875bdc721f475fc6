# round 6, call 17: the final build again (call 16's suite stopped at one in-process peer-exchange timeout,
# recorded in profiles/r06_gpu_tests_c16_peer_timeout.log and DESIGN §6.2) -- the whole GPU suite, smoke,
# and the driver's bench command
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
tools/gpu_steps.sh \
  700 r6/c17_tests.log 'python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread' \
  120 r6/c17_smoke.log 'python -c "import __graft_entry__ as g; g.smoke()"' \
  600 r6/c17_bench.log 'python bench.py --steps 20 --warmup 5 > gpurun_out/r6/c17_bench_steps20_warmup5.json'
