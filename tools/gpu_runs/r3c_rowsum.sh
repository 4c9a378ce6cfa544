# generalised bias fold (wide slices, split-K partials, LDS accumulators): GEMM tests, benches
set -e
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "fused_bias or schedules or layouts or split_k or wgrad or linear" > gpurun_out/rs_tests.log 2>&1
for i in 1 2; do
  MIPIPE_FUSE_BIAS=0 timeout -k 10 300 python -u bench.py --config gpt2_xl --steps 3 --warmup 2 --no-bubble > gpurun_out/rs_gpt0_$i.log 2>&1
  MIPIPE_FUSE_BIAS=1 timeout -k 10 300 python -u bench.py --config gpt2_xl --steps 3 --warmup 2 --no-bubble > gpurun_out/rs_gpt1_$i.log 2>&1
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/rs_enc.log 2>&1
