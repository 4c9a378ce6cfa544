#!/bin/bash
# Staged-layout EXTRA epilogue (dropout / aux): GEMM tests + screens, epilogue probe, GPT-2-XL + enc12 benches.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "linear or gemm or dropout or gelu or act or x_transposed or feedforward or bias" > gpurun_out/b6_tests.log 2>&1 || { tail -40 gpurun_out/b6_tests.log; exit 1; }
tail -1 gpurun_out/b6_tests.log
timeout -k 10 300 python -u tools/gemm_round_screen.py 20 > gpurun_out/round_screen6.txt 2>&1 || { tail -20 gpurun_out/round_screen6.txt; exit 1; }
echo "round screen: $(grep -c 'all identical' gpurun_out/round_screen6.txt)/20 identical"
timeout -k 10 200 python -u tools/gemm_seq_screen.py 30 2>&1 | tail -4
timeout -k 10 200 python -u tools/epilogue_cost_probe.py > gpurun_out/epilogue_probe6.txt 2>&1; cat gpurun_out/epilogue_probe6.txt
val() { grep -o '"value": [0-9.]*' "$1" | head -1; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --config gpt2_xl --steps 4 --warmup 2 --no-bubble > gpurun_out/gpt6_$i.log 2>&1 || { tail -20 gpurun_out/gpt6_$i.log; exit 1; }
  echo "gpt2_xl run $i: $(val gpurun_out/gpt6_$i.log)"
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-bubble > gpurun_out/enc6_$i.log 2>&1 || { tail -20 gpurun_out/enc6_$i.log; exit 1; }
  echo "enc12 run $i: $(val gpurun_out/enc6_$i.log)"
done
