#!/bin/bash
# GPT-2-XL weight-gradient flush: split-K factor sweep, then the flush-time x^T arms (r4_b20.sh).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u tools/splitk_probe.py 18432 4 > gpurun_out/b21_splitk.log 2>&1 || { tail -20 gpurun_out/b21_splitk.log; exit 1; }
grep -v amdgpu.ids gpurun_out/b21_splitk.log
bash tools/gpu_runs/r4_b20.sh
