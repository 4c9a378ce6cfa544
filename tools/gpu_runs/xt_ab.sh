#!/bin/bash
# x^T emission + transposed weight-gradient GEMM: GEMM tests, then a same-box bench A/B
# (MIPIPE_WGRAD_XT=0: the round-3 path), arms alternated.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "gemm or wgrad or linear or cross_entropy or x_transposed" > gpurun_out/xt_tests.log 2>&1 || { tail -30 gpurun_out/xt_tests.log; exit 1; }
tail -2 gpurun_out/xt_tests.log
for i in 1 2; do
  for xt in 0 1; do
    MIPIPE_WGRAD_XT=$xt timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-bubble > gpurun_out/xt_bench${xt}_$i.log 2>&1 || { tail -20 gpurun_out/xt_bench${xt}_$i.log; exit 1; }
    echo "xt=$xt run $i: $(grep -o '"value": [0-9.]*' gpurun_out/xt_bench${xt}_$i.log) $(grep -o '"peak_hbm_gib[^]]*' gpurun_out/xt_bench${xt}_$i.log | head -c 80)"
  done
done
