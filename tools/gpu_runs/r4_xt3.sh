#!/bin/bash
# flush-time transpose for the transposed weight-gradient GEMM: tests, transpose bandwidth, bench A/B, profile.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "transpose or xt_path or wgrad_xt or x_transposed or activation_backward or act_fold or gelu_saved or feedforward" > gpurun_out/xt3_tests.log 2>&1 || { tail -40 gpurun_out/xt3_tests.log; exit 1; }
tail -2 gpurun_out/xt3_tests.log
timeout -k 10 120 python -u tools/transpose_bw.py 2>&1 | tee gpurun_out/transpose_bw.txt
val() { grep -o '"value": [0-9.]*' "$1" | head -1; }
for i in 1 2; do
  for xt in 0 auto; do
    MIPIPE_WGRAD_XT=$xt timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-bubble > gpurun_out/xt3_bench${xt}_$i.log 2>&1 || { tail -20 gpurun_out/xt3_bench${xt}_$i.log; exit 1; }
    echo "enc12 xt=$xt run $i: $(val gpurun_out/xt3_bench${xt}_$i.log) $(grep -o '"peak_hbm_gib_per_gpu": \[[0-9., ]*\]' gpurun_out/xt3_bench${xt}_$i.log)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_xt3 -o run -- python3 bench.py --steps 4 --warmup 2 --no-bubble > gpurun_out/prof_xt3.log 2>&1 || { tail -5 gpurun_out/prof_xt3.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof_xt3/run_results.db 40 --by-grid 2>&1 | grep "gemm256\|transpose" | head -14
