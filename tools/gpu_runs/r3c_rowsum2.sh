# bias fold with division-free slice mapping: tests, then same-box A/B (MIPIPE_FUSE_BIAS) on both PP=1 configs
set -e
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "fused_bias or schedules or wgrad or linear" > gpurun_out/rs2_tests.log 2>&1
for i in 1 2; do
  MIPIPE_FUSE_BIAS=0 timeout -k 10 200 python -u bench.py --steps 8 --warmup 3 --no-bubble > gpurun_out/rs2_enc0_$i.log 2>&1
  MIPIPE_FUSE_BIAS=1 timeout -k 10 200 python -u bench.py --steps 8 --warmup 3 --no-bubble > gpurun_out/rs2_enc1_$i.log 2>&1
  MIPIPE_FUSE_BIAS=0 timeout -k 10 300 python -u bench.py --config gpt2_xl --steps 3 --warmup 2 --no-bubble > gpurun_out/rs2_gpt0_$i.log 2>&1
  MIPIPE_FUSE_BIAS=1 timeout -k 10 300 python -u bench.py --config gpt2_xl --steps 3 --warmup 2 --no-bubble > gpurun_out/rs2_gpt1_$i.log 2>&1
done
