#!/bin/bash
# Round 5: the bench's looping PP=4 path (chunks 16, 'never', v / split from the plan) as 4 ranks sharing one
# MI355X over the IPC links -- a functional rehearsal of the driver's N=4 run (time-sliced: NOT a throughput number).
# Micro-batch 32 to fit 4 ranks on one GPU; progress lines every step.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 MIPIPE_BENCH_PROGRESS=1 MIPIPE_IPC_DEBUG=1
timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29617 bench.py --gpus 4 --shared-gpu --micro-batch 32 --steps 2 --warmup 1 --no-bubble --watchdog 120 > gpurun_out/pp4_shared.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 20; echo "[$(date +%T)] $(grep -c '' gpurun_out/pp4_shared.log) lines; last: $(grep '^\[bench' gpurun_out/pp4_shared.log | tail -1)" >> gpurun_out/pp4_heartbeat.txt; done
wait $pid
rc=$?
cat gpurun_out/pp4_heartbeat.txt | tail -5
[ $rc -eq 0 ] || { grep "mipipe ipc\|^\[bench" gpurun_out/pp4_shared.log | tail -40; exit $rc; }
grep '"metric"' gpurun_out/pp4_shared.log | cut -c1-1200
