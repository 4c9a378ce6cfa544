#!/bin/bash
# GPT-2-XL A/B (GELU fold only without dropout), IPC engine A/B on the 2-rank shared-GPU rehearsal,
# engine-context measured planning vs analytic on the PP=8 rank emulations.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
bash tools/gpu_runs/r4_gpt.sh || exit 1
val() { grep -o '"value": [0-9.]*' "$1" | head -1; }
for i in 1 2; do
  for eng in sdma inline; do
    MIPIPE_IPC_ENGINE=$eng GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port $((29600 + i)) bench.py --gpus 2 --shared-gpu --config enc12_d4096 --num-layers 4 \
      --micro-batch 16 --chunks 8 --steps 6 --warmup 2 --no-bubble > gpurun_out/shared_${eng}_$i.log 2>&1 || { tail -20 gpurun_out/shared_${eng}_$i.log; exit 1; }
    echo "shared-gpu 2 ranks engine=$eng run $i: $(val gpurun_out/shared_${eng}_$i.log)"
  done
done
bash tools/gpu_runs/r4_plan.sh
