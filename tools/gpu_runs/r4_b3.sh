#!/bin/bash
# GPT-2-XL A/B + profile, IPC latency incl. the inline engine, measured-cost planning emulation.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pipeline.py -k "ipc" > gpurun_out/ipc_tests3.log 2>&1 || { tail -30 gpurun_out/ipc_tests3.log; exit 1; }
tail -1 gpurun_out/ipc_tests3.log
bash tools/gpu_runs/r4_gpt.sh || exit 1
GPU_MAX_HW_QUEUES=16 timeout -k 10 400 python -u tools/ipc_bw.py --iters 20 > gpurun_out/ipc_bw3.txt 2>&1 || { tail -20 gpurun_out/ipc_bw3.txt; exit 1; }
grep -v "^\[rank .*MiB$\|Gloo\|socket\|it [0-9]$" gpurun_out/ipc_bw3.txt
bash tools/gpu_runs/r4_plan.sh
