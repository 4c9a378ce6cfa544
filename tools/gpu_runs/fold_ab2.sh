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
# micro-batch sizing for the 1600-wide GEMMs (M = mb x 1024 -> 256-row tiles x 7 column tiles per round)
for mb in 9 12; do
  timeout -k 10 300 python -u bench.py --config gpt2_xl --micro-batch $mb --steps 4 --warmup 2 --no-bubble > gpurun_out/fb_gpt_mb${mb}.log 2>&1
done
# GEMM schedule A/B (ping-pong vs B staged two tiles ahead) + a correctness pass of the GEMM tests under the new schedule
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
MIPIPE_GEMM_SCHED=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "linear or gemm or vocab or fold" > gpurun_out/sab_tests.log 2>&1
timeout -k 10 400 python -u tools/gemm_sched_ab.py 2 3 > gpurun_out/sched_ab.log 2>&1
