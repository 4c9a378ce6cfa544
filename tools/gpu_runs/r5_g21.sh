#!/bin/bash
# Round 5: 8- vs 4-wave GEMM block SUSTAINED at the power cap; then the except_last rehearsal (r5_g20.sh).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/gemm_clock_probe.py --waves > gpurun_out/gemm_waves_sustained.txt 2>&1 || { tail -20 gpurun_out/gemm_waves_sustained.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/gemm_waves_sustained.txt
bash tools/gpu_runs/r5_g20.sh
