# round 6, call 19: the policy gradient's LogStd sum and finish in one launch (no collective): the whole GPU
# suite, an interleaved A/B of whole updates before (up0) and after (up1), then the driver's bench command
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
V=trpo-robot-control_amd/lib/variants
tools/gpu_steps.sh \
  700 r6/c19_tests.log 'python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread' \
  400 r6/c19_ab.log "ROUNDS=7 timeout -k 5 300 python tools/ab_update.py $V/up0.so $V/up1.so" \
  120 r6/c19_smoke.log 'python -c "import __graft_entry__ as g; g.smoke()"' \
  600 r6/c19_bench.log 'python bench.py --steps 20 --warmup 5 > gpurun_out/r6/c19_bench_steps20_warmup5.json'
