#!/bin/bash
# Flush-time x^T without the tile floor (GPT-2-XL fc1 now transposed, its bias folded): tests + GPT-2-XL A/B.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_pipeline.py -k "xt or wgrad or linear or gpt or bit" > gpurun_out/b22_tests.log 2>&1 || { tail -30 gpurun_out/b22_tests.log; exit 1; }
tail -1 gpurun_out/b22_tests.log
val() { grep -o '"value": [0-9.]*' "$1" | head -1; }
for i in 1 2; do
  for arm in old new; do
    envs=""; [ $arm = old ] && envs="MIPIPE_WGRAD_XT_MIN_TILES=512"
    env $envs timeout -k 10 300 python -u bench.py --config gpt2_xl --steps 4 --warmup 2 --no-bubble > gpurun_out/b22_gpt_${arm}_$i.log 2>&1 || { tail -20 gpurun_out/b22_gpt_${arm}_$i.log; exit 1; }
    echo "gpt2_xl $arm run $i: $(val gpurun_out/b22_gpt_${arm}_$i.log)"
  done
done
