#!/bin/bash
# flush-time transpose A/B + stream-ordered IPC latency (GPU-paced) + shared-GPU timeline.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_runs/r4_xt3.sh || exit 1
export PYTHONUNBUFFERED=1 GPU_MAX_HW_QUEUES=16
timeout -k 10 400 python -u tools/ipc_bw.py --iters 20 > gpurun_out/ipc_bw2.txt 2>&1 || { tail -20 gpurun_out/ipc_bw2.txt; exit 1; }
grep -v "^\[rank .*MiB$" gpurun_out/ipc_bw2.txt
timeout -k 10 400 python -u tools/profile_ranks.py --nproc 2 --out gpurun_out/tl3 -- --shared-gpu --config enc12_d4096 --num-layers 4 --micro-batch 16 --chunks 8 --steps 2 --warmup 1 --no-bubble > gpurun_out/tl3.txt 2>&1 || { tail -30 gpurun_out/tl3.txt; exit 1; }
python3 tools/engine_timeline.py "gpurun_out/tl3/rank*/rank_results.db"
