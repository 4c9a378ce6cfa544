#!/bin/bash
# I-contiguous staging window closed (A in 128-row halves, B in three buffers): GEMM tests, race screens,
# enc12 / GPT-2-XL A/B vs HEAD.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py > gpurun_out/b16_tests.log 2>&1 || { tail -30 gpurun_out/b16_tests.log; exit 1; }
tail -1 gpurun_out/b16_tests.log
timeout -k 10 300 python -u tools/gemm_race_screen.py 4096 4800 1600 20 > gpurun_out/b16_race1.log 2>&1 || { tail -20 gpurun_out/b16_race1.log; exit 1; }
timeout -k 10 300 python -u tools/gemm_race_screen.py 8192 4096 4096 10 > gpurun_out/b16_race2.log 2>&1 || { tail -20 gpurun_out/b16_race2.log; exit 1; }
grep -c "0/" gpurun_out/b16_race1.log gpurun_out/b16_race2.log; grep -v " 0/" gpurun_out/b16_race1.log gpurun_out/b16_race2.log || true
val() { grep -o '"value": [0-9.]*' "$1" | head -1; }
for i in 1 2; do
  for arm in old new; do
    b=bench.py; [ $arm = old ] && b=ab_old/bench.py
    timeout -k 10 300 python -u $b --steps 10 --warmup 3 --no-bubble > gpurun_out/b16_enc_${arm}_$i.log 2>&1 || { tail -20 gpurun_out/b16_enc_${arm}_$i.log; exit 1; }
    echo "enc12 $arm run $i: $(val gpurun_out/b16_enc_${arm}_$i.log)"
  done
done
for arm in old new; do
  b=bench.py; [ $arm = old ] && b=ab_old/bench.py
  timeout -k 10 300 python -u $b --config gpt2_xl --steps 4 --warmup 2 --no-bubble > gpurun_out/b16_gpt_${arm}.log 2>&1 || { tail -20 gpurun_out/b16_gpt_${arm}.log; exit 1; }
  echo "gpt2_xl $arm: $(val gpurun_out/b16_gpt_${arm}.log)"
done
