# half-tile ping-pong (schedule 5) vs the default (4): GEMM tests, in-process shape A/B, enc12 bench A/B
set -e
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "schedules or layouts or split_k or round_launches" > gpurun_out/s5_tests.log 2>&1
timeout -k 10 400 python -u tools/gemm_sched_ab.py 4 5 > gpurun_out/s5_ab.log 2>&1
for i in 1 2; do
  MIPIPE_GEMM_SCHED=4 timeout -k 10 200 python -u bench.py --steps 8 --warmup 3 --no-bubble > gpurun_out/s5_bench4_$i.log 2>&1
  MIPIPE_GEMM_SCHED=5 timeout -k 10 200 python -u bench.py --steps 8 --warmup 3 --no-bubble > gpurun_out/s5_bench5_$i.log 2>&1
done
