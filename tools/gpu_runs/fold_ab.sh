# A/B of the MLP activation-backward fold (MIPIPE_FOLD_ACT) on the PP=1 benches, arms alternated;
# then the GPT-2-XL PP=1 bench and the Adam tests.
set -e
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "adam or fold" > gpurun_out/fa_tests.log 2>&1
for r in 1 2; do
  for f in 1 0; do
    MIPIPE_FOLD_ACT=$f timeout -k 10 240 python -u bench.py --steps 6 --warmup 2 --no-bubble > gpurun_out/fa_enc_f${f}_r${r}.log 2>&1
  done
done
for f in 1 0; do
  MIPIPE_FOLD_ACT=$f timeout -k 10 300 python -u bench.py --config gpt2_xl --steps 4 --warmup 2 --no-bubble > gpurun_out/fa_gpt_f${f}.log 2>&1
done
