#!/bin/bash
# Round 5: the bench's full PP=8 path (config #3: enc12, chunks 32, micro-batch 64, except_last, looping plan, split
# head) as 8 ranks sharing one MI355X over the IPC links -- a functional rehearsal of the driver's N=8 run (time-sliced
# on one GPU: NOT a throughput number).  Micro-batch 32: at 64 the 8 ranks (33 GB each + 8 GB of IPC rings) exceed one
# GPU's 288 GB -- on the 8-GPU node each rank has its own.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 MIPIPE_BENCH_PROGRESS=1
timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29615 bench.py --gpus 8 --shared-gpu --micro-batch 32 --steps 2 --warmup 1 --no-bubble > gpurun_out/pp8_shared.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 20; echo "[$(date +%T)] $(grep '^\[bench' gpurun_out/pp8_shared.log | tail -1)" >> gpurun_out/pp8_heartbeat.txt; done
wait $pid || { tail -5 gpurun_out/pp8_heartbeat.txt; grep -v "amdgpu.ids\|^\[W\|^W20" gpurun_out/pp8_shared.log | tail -30; exit 1; }
grep '"metric"' gpurun_out/pp8_shared.log | cut -c1-1500
