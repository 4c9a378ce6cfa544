#!/bin/bash
# Stream-ordered IPC links: GPU tests, bandwidth / latency table, 2-rank shared-GPU timeline.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 GPU_MAX_HW_QUEUES=16
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pipeline.py -k "ipc" > gpurun_out/ipc_tests.log 2>&1 || { tail -40 gpurun_out/ipc_tests.log; exit 1; }
tail -2 gpurun_out/ipc_tests.log
timeout -k 10 300 python -u tools/ipc_bw.py --iters 20 > gpurun_out/ipc_bw.txt 2>&1 || { tail -20 gpurun_out/ipc_bw.txt; exit 1; }
grep -v "^\[rank" gpurun_out/ipc_bw.txt
timeout -k 10 400 python -u tools/profile_ranks.py --nproc 2 --out gpurun_out/tl2 -- --shared-gpu --config enc12_d4096 --num-layers 4 --micro-batch 16 --chunks 8 --steps 2 --warmup 1 --no-bubble > gpurun_out/tl2.txt 2>&1 || { tail -30 gpurun_out/tl2.txt; exit 1; }
grep -v "^\[" gpurun_out/tl2.txt | tail -12
