#!/bin/bash
# The A-side bias fold for every both-I-contiguous weight-gradient grid (under 16 tile columns, split-K): tests,
# GPT-2-XL A/B (its qkv / out / fc2 bias column-sum passes go away), enc12 check.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_pipeline.py -k "wgrad or gemm or linear or bias or gpt or bit" > gpurun_out/b24_tests.log 2>&1 || { tail -30 gpurun_out/b24_tests.log; exit 1; }
tail -1 gpurun_out/b24_tests.log
val() { grep -o '"value": [0-9.]*' "$1" | head -1; }
for i in 1 2; do
  for arm in old new; do
    b=bench.py; [ $arm = old ] && b=ab_old/bench.py
    timeout -k 10 300 python -u $b --config gpt2_xl --steps 4 --warmup 2 --no-bubble > gpurun_out/b24_gpt_${arm}_$i.log 2>&1 || { tail -20 gpurun_out/b24_gpt_${arm}_$i.log; exit 1; }
    echo "gpt2_xl $arm run $i: $(val gpurun_out/b24_gpt_${arm}_$i.log)"
  done
done
for arm in old new; do
  b=bench.py; [ $arm = old ] && b=ab_old/bench.py
  timeout -k 10 300 python -u $b --steps 10 --warmup 3 --no-bubble > gpurun_out/b24_enc_${arm}.log 2>&1 || { tail -20 gpurun_out/b24_enc_${arm}.log; exit 1; }
  echo "enc12 $arm: $(val gpurun_out/b24_enc_${arm}.log)"
done
