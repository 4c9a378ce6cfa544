# fold + fp32-attention tests, then GPT-2-XL PP=1 A/B of the activation fold (arms alternated).
set -e
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_fp32.py -k "fold or attention_f32 or learned or vocab" > gpurun_out/fb_tests.log 2>&1
for r in 1 2; do
  for f in 1 0; do
    MIPIPE_FOLD_ACT=$f timeout -k 10 300 python -u bench.py --config gpt2_xl --steps 4 --warmup 2 --no-bubble > gpurun_out/fb_gpt_f${f}_r${r}.log 2>&1
  done
done
