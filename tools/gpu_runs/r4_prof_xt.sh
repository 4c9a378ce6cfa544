#!/bin/bash
# GELU epilogue mismatch screen, then kernel traces of the enc12 PP=1 bench with and without the x^T path.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/gemm_gelu_screen.py 15 > gpurun_out/gelu_screen.txt 2>&1; cat gpurun_out/gelu_screen.txt
for xt in 1 0; do
  MIPIPE_WGRAD_XT=$xt timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_xt$xt -o run -- python3 bench.py --steps 4 --warmup 2 --no-bubble > gpurun_out/prof_xt$xt.log 2>&1 || { tail -5 gpurun_out/prof_xt$xt.log; exit 1; }
  f=$(ls gpurun_out/prof_xt$xt/*/run_kernel_stats.csv gpurun_out/prof_xt$xt/run_kernel_stats.csv 2>/dev/null | head -1)
  echo "== xt=$xt $f"; python3 tools/prof_summary.py "$f" 14
done
