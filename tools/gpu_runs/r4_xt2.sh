#!/bin/bash
# x^T path after the register fixes: tests, round screen, same-box bench A/B, kernel profile of the x^T arm.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "gemm or wgrad or linear or cross_entropy or x_transposed" > gpurun_out/xt_tests.log 2>&1 || { tail -40 gpurun_out/xt_tests.log; exit 1; }
tail -2 gpurun_out/xt_tests.log
timeout -k 10 200 python -u tools/gemm_seq_screen.py 40 > gpurun_out/seq_screen.txt 2>&1; cat gpurun_out/seq_screen.txt
timeout -k 10 300 python -u tools/gemm_round_screen.py 30 > gpurun_out/round_screen.txt 2>&1 || { cat gpurun_out/round_screen.txt; exit 1; }
echo "round screen: $(grep -c 'all identical' gpurun_out/round_screen.txt)/30 identical"; grep -v "all identical" gpurun_out/round_screen.txt | head -4
val() { grep -o '"value": [0-9.]*' "$1" | head -1; }
for i in 1 2; do
  for xt in 0 1; do
    MIPIPE_WGRAD_XT=$xt timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-bubble > gpurun_out/xt_bench${xt}_$i.log 2>&1 || { tail -20 gpurun_out/xt_bench${xt}_$i.log; exit 1; }
    echo "enc12 xt=$xt run $i: $(val gpurun_out/xt_bench${xt}_$i.log) $(grep -o '"peak_hbm_gib_per_gpu": \[[0-9., ]*\]' gpurun_out/xt_bench${xt}_$i.log)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_xt1b -o run -- python3 bench.py --steps 4 --warmup 2 --no-bubble > gpurun_out/prof_xt1b.log 2>&1 || { tail -5 gpurun_out/prof_xt1b.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof_xt1b/run_results.db 40 --by-grid 2>&1 | grep gemm256 | head -12
