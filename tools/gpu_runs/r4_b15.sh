#!/bin/bash
# Fast-erf GELU in the elementwise kernels: activation tests; GPT-2-XL A/B vs HEAD; GELU backward kernel time.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_fp32.py -k "gelu or act or bias or linear or feedforward" > gpurun_out/b15_tests.log 2>&1 || { tail -30 gpurun_out/b15_tests.log; exit 1; }
tail -1 gpurun_out/b15_tests.log
val() { grep -o '"value": [0-9.]*' "$1" | head -1; }
for i in 1 2; do
  for arm in old new; do
    b=bench.py; [ $arm = old ] && b=ab_old/bench.py
    timeout -k 10 300 python -u $b --config gpt2_xl --steps 4 --warmup 2 --no-bubble > gpurun_out/b15_gpt_${arm}_$i.log 2>&1 || { tail -20 gpurun_out/b15_gpt_${arm}_$i.log; exit 1; }
    echo "gpt2_xl $arm run $i: $(val gpurun_out/b15_gpt_${arm}_$i.log)"
  done
done
