#!/bin/bash
# Intermittent-race screen: forward GEMM with / without x^T emission, then the b10 batch.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/emit_screen.py 60 > gpurun_out/emit_screen.txt 2>&1; tail -12 gpurun_out/emit_screen.txt
timeout -k 10 300 python -u tools/gemm_round_screen.py 20 > gpurun_out/round_screen11.txt 2>&1; echo "round screen: $(grep -c 'all identical' gpurun_out/round_screen11.txt)/20 identical"
