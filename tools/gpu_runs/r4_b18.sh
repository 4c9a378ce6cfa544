#!/bin/bash
# bias+activation kernels: all loads of a 4-row tile first; GELU' with one exp.  Tests, kernel A/B, GPT-2-XL A/B.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_fp32.py -k "gelu or act or bias or dropout or linear or feedforward or transformer" > gpurun_out/b18_tests.log 2>&1 || { tail -30 gpurun_out/b18_tests.log; exit 1; }
tail -1 gpurun_out/b18_tests.log
for i in 1 2; do
  timeout -k 10 200 python -u tools/bias_act_ab.py ab_old old > gpurun_out/b18_ba_old_$i.log 2>&1 || { tail -20 gpurun_out/b18_ba_old_$i.log; exit 1; }
  timeout -k 10 200 python -u tools/bias_act_ab.py . new > gpurun_out/b18_ba_new_$i.log 2>&1 || { tail -20 gpurun_out/b18_ba_new_$i.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/b18_ba_old_$i.log gpurun_out/b18_ba_new_$i.log
done
timeout -k 10 100 python -u tools/bias_act_ab.py --compare old new
val() { grep -o '"value": [0-9.]*' "$1" | head -1; }
for i in 1 2; do
  for arm in old new; do
    b=bench.py; [ $arm = old ] && b=ab_old/bench.py
    timeout -k 10 300 python -u $b --config gpt2_xl --steps 4 --warmup 2 --no-bubble > gpurun_out/b18_gpt_${arm}_$i.log 2>&1 || { tail -20 gpurun_out/b18_gpt_${arm}_$i.log; exit 1; }
    echo "gpt2_xl $arm run $i: $(val gpurun_out/b18_gpt_${arm}_$i.log)"
  done
done
