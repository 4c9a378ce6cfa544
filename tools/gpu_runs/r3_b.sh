# schedule tests (incl. the new default), dact epilogue probe, enc12 + GPT-2-XL benches on the new default schedule
set -e
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "schedules" > gpurun_out/rb_tests.log 2>&1
timeout -k 10 200 python -u tools/gemm_dact_probe.py > gpurun_out/dact_probe.log 2>&1
timeout -k 10 240 python -u bench.py --steps 8 --warmup 3 --no-bubble > gpurun_out/rb_enc.log 2>&1
for mb in 9 18; do
  timeout -k 10 400 python -u bench.py --config gpt2_xl --micro-batch $mb --steps 4 --warmup 2 --no-bubble > gpurun_out/rb_gpt_mb${mb}.log 2>&1
done
