#!/bin/bash
# LayerNorm forward (one row per block): gamma / beta loaded with the row, one barrier per reduction (2 instead of 4).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_fp32.py -k "layernorm or layer_norm or ln or transformer" > gpurun_out/b23_tests.log 2>&1 || { tail -30 gpurun_out/b23_tests.log; exit 1; }
tail -1 gpurun_out/b23_tests.log
for i in 1 2; do
  timeout -k 10 200 python -u tools/ln_fwd_ab.py ab_old old > gpurun_out/b23_ln_old_$i.log 2>&1 || { tail -20 gpurun_out/b23_ln_old_$i.log; exit 1; }
  timeout -k 10 200 python -u tools/ln_fwd_ab.py . new > gpurun_out/b23_ln_new_$i.log 2>&1 || { tail -20 gpurun_out/b23_ln_new_$i.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/b23_ln_old_$i.log gpurun_out/b23_ln_new_$i.log
done
timeout -k 10 100 python -u tools/ln_fwd_ab.py --compare old new
val() { grep -o '"value": [0-9.]*' "$1" | head -1; }
for i in 1 2; do
  for arm in old new; do
    b=bench.py; [ $arm = old ] && b=ab_old/bench.py
    timeout -k 10 300 python -u $b --steps 10 --warmup 3 --no-bubble > gpurun_out/b23_enc_${arm}_$i.log 2>&1 || { tail -20 gpurun_out/b23_enc_${arm}_$i.log; exit 1; }
    echo "enc12 $arm run $i: $(val gpurun_out/b23_enc_${arm}_$i.log)"
  done
done
