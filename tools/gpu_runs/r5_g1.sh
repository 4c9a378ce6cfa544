#!/bin/bash
# Round 5 call: 4-wave GEMM harness + product A/B, then the bench + hipBLASLt id + CU-hold probe.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 120 tools/micro/bin/gemm4w 8192 4096 > gpurun_out/gemm4w.txt 2>&1 || { cat gpurun_out/gemm4w.txt; exit 1; }
cat gpurun_out/gemm4w.txt
timeout -k 10 300 python -u tools/gemm_waves_ab.py 8192 > gpurun_out/gemm_waves_ab.txt 2>&1 || { cat gpurun_out/gemm_waves_ab.txt; exit 1; }
cat gpurun_out/gemm_waves_ab.txt
bash tools/gpu_runs/r5_hold.sh
