#!/bin/bash
# GPT-2-XL weight-gradient layouts at the real flush K (4 micro-batches x 18432 tokens).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/wgrad_layout_probe.py 73728 gpt2xl > gpurun_out/b19_probe.log 2>&1 || { tail -20 gpurun_out/b19_probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/b19_probe.log
timeout -k 10 300 python -u tools/wgrad_layout_probe.py 18432 gpt2xl > gpurun_out/b19_probe2.log 2>&1 || { tail -20 gpurun_out/b19_probe2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/b19_probe2.log
