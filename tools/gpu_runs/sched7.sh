# GEMM main-loop schedules 4 (ping-pong + B lead), 5 (half-tile), 6 (half-tile on KC layouts, 4 on wgrad), 7 (whole-tile)
set -e
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "schedules or fused_bias or layouts" > gpurun_out/s7_tests.log 2>&1
timeout -k 10 500 python -u tools/gemm_sched_ab.py 4 5 7 > gpurun_out/s7_ab.log 2>&1
timeout -k 10 300 python -u tools/wgrad_probe.py 4 5 7 > gpurun_out/s7_wgrad.log 2>&1 || true
for i in 1 2; do
  for s in 4 6 7; do
    MIPIPE_GEMM_SCHED=$s timeout -k 10 200 python -u bench.py --steps 8 --warmup 3 --no-bubble > gpurun_out/s7_bench${s}_$i.log 2>&1
  done
done
