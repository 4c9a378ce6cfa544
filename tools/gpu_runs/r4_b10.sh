#!/bin/bash
# K < 4096 multi-round GEMMs in one launch: GEMM tests, GPT-2-XL / enc12 benches, final GPT-2-XL kernel profile.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "gemm or linear or wgrad" > gpurun_out/b10_tests.log 2>&1 || { tail -30 gpurun_out/b10_tests.log; exit 1; }
tail -1 gpurun_out/b10_tests.log
val() { grep -o '"value": [0-9.]*' "$1" | head -1; }
for i in 1 2; do
  for r in 2 1; do
    MIPIPE_GEMM_ROUNDS=$r timeout -k 10 300 python -u bench.py --config gpt2_xl --steps 4 --warmup 2 --no-bubble > gpurun_out/b10_gpt_r${r}_$i.log 2>&1 || { tail -20 gpurun_out/b10_gpt_r${r}_$i.log; exit 1; }
    echo "gpt2_xl rounds=$r run $i: $(val gpurun_out/b10_gpt_r${r}_$i.log) $(grep -o '"peak_hbm_gib_per_gpu": \[[0-9., ]*\]' gpurun_out/b10_gpt_r${r}_$i.log)"
  done
done
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/b10_enc.log 2>&1 || { tail -20 gpurun_out/b10_enc.log; exit 1; }
echo "enc12 default: $(val gpurun_out/b10_enc.log) $(grep -o '"bubble_pct": [0-9.]*' gpurun_out/b10_enc.log)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gpt10 -o run -- python3 bench.py --config gpt2_xl --steps 2 --warmup 1 --no-bubble > gpurun_out/prof_gpt10.log 2>&1 || { tail -5 gpurun_out/prof_gpt10.log; exit 1; }
echo "gpt under rocprof: $(val gpurun_out/prof_gpt10.log)"
python3 tools/prof_summary.py gpurun_out/prof_gpt10/run_results.db 24 2>&1 | head -28
