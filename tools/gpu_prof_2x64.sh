export TMPDIR=/tmp
mkdir -p gpurun_out/p2x64
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p2x64 -o run -- python3 tools/cg_only.py 2x64 50000 20 > gpurun_out/p2x64/run.log 2>&1
