#!/bin/bash
# GEMM PP=4 schedule with group 1's restaging behind the interval barrier: tests, race screens, same-box A/B vs HEAD.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "gemm or linear or wgrad or x_transposed" > gpurun_out/b12_tests.log 2>&1 || { tail -30 gpurun_out/b12_tests.log; exit 1; }
tail -1 gpurun_out/b12_tests.log
timeout -k 10 300 python -u tools/gemm_round_screen.py 20 > gpurun_out/round_screen12.txt 2>&1; echo "round screen: $(grep -c 'all identical' gpurun_out/round_screen12.txt)/20 identical"
timeout -k 10 200 python -u tools/gemm_seq_screen.py 30 2>&1 | tail -4
timeout -k 10 300 python -u tools/emit_screen.py 40 2>&1 | tail -2
timeout -k 10 300 python -u tools/emit_screen.py 40 2048 9000 512 2>&1 | tail -2
val() { grep -o '"value": [0-9.]*' "$1" | head -1; }
for i in 1 2; do
  for arm in old new; do
    b=bench.py; [ $arm = old ] && b=ab_old/bench.py
    timeout -k 10 200 python -u $b --steps 10 --warmup 3 --no-bubble > gpurun_out/b12_enc_${arm}_$i.log 2>&1 || { tail -20 gpurun_out/b12_enc_${arm}_$i.log; exit 1; }
    echo "enc12 $arm run $i: $(val gpurun_out/b12_enc_${arm}_$i.log)"
  done
done
for i in 1 2; do
  for arm in old new; do
    b=bench.py; [ $arm = old ] && b=ab_old/bench.py
    timeout -k 10 300 python -u $b --config gpt2_xl --steps 4 --warmup 2 --no-bubble > gpurun_out/b12_gpt_${arm}_$i.log 2>&1 || { tail -20 gpurun_out/b12_gpt_${arm}_$i.log; exit 1; }
    echo "gpt2_xl $arm run $i: $(val gpurun_out/b12_gpt_${arm}_$i.log)"
  done
done
