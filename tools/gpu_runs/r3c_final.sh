# round-3 final tree: driver-style smoke and default bench
set -e
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/final_bench.log 2>&1
