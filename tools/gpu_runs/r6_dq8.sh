#!/bin/bash
# Long-sequence dQ with 32-query waves in 8-wave (MIPIPE_ATTN_DQ8=8) or 4-wave (=4) blocks vs the 4-wave kernel of
# 64-query waves (=0): numerics, kernel time at GPT-2-XL's shape, then the GPT-2-XL step.  Arms interleaved.
set -o pipefail
mkdir -p gpurun_out/dq8
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
for arm in 8 4; do
  MIPIPE_ATTN_DQ8=$arm timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu -k "attention" > gpurun_out/dq8/tests_$arm.log 2>&1 || { tail -30 gpurun_out/dq8/tests_$arm.log; exit 1; }
  echo "dq8=$arm tests: $(tail -1 gpurun_out/dq8/tests_$arm.log)"
done
for i in 1 2; do
  for arm in 0 8 4; do
    MIPIPE_ATTN_DQ8=$arm timeout -k 10 120 python -u tools/bench_attn.py 18 1024 25 64 causal 0.1 2>&1 | grep "kernels=1" | sed "s/^/dq8=$arm $i /" || exit 1
  done
done
for i in 1 2; do
  for arm in 0 8 4; do
    timeout -k 10 400 env MIPIPE_ATTN_DQ8=$arm python -u bench.py --config gpt2_xl --steps 10 --warmup 3 --no-bubble > gpurun_out/dq8/g_${arm}_$i.log 2>&1 || { tail -20 gpurun_out/dq8/g_${arm}_$i.log; exit 1; }
    echo "dq8=$arm $i gpt2_xl: $(grep -o '"value": [0-9.]*' gpurun_out/dq8/g_${arm}_$i.log) $(grep -o '"gfxclk_mhz": {"mean": [0-9.]*' gpurun_out/dq8/g_${arm}_$i.log)"
  done
done
