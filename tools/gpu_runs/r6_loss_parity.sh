#!/bin/bash
# Loss parity PP=1 vs PP=2 (two ranks sharing one MI355X, IPC links) at the SAME micro-batch, chunks and steps:
# the engine's multi-rank step must train the same model the same way.  enc12 (never) and GPT-2-XL (always).
set -o pipefail
mkdir -p gpurun_out/parity
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
loss() { python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print(sys.argv[2], 'loss', d['loss'], 'tok/s', d['value'], d['config']['parallelism'], d['config']['chunks'], d['config']['micro_batch'], d['config']['checkpoint'])" "$1" "$2"; }
E="--micro-batch 32 --chunks 8 --steps 3 --warmup 1 --no-bubble"
timeout -k 10 300 python -u bench.py $E > gpurun_out/parity/e1.log 2>&1 || { tail -20 gpurun_out/parity/e1.log; exit 1; }
loss gpurun_out/parity/e1.log enc12_pp1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29741 bench.py --gpus 2 --shared-gpu $E > gpurun_out/parity/e2.log 2>&1 || { tail -20 gpurun_out/parity/e2.log; exit 1; }
loss gpurun_out/parity/e2.log enc12_pp2
G="--config gpt2_xl --micro-batch 4 --chunks 8 --steps 3 --warmup 1 --no-bubble"
timeout -k 10 300 python -u bench.py $G > gpurun_out/parity/g1.log 2>&1 || { tail -20 gpurun_out/parity/g1.log; exit 1; }
loss gpurun_out/parity/g1.log gpt2_pp1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29743 bench.py --gpus 2 --shared-gpu $G > gpurun_out/parity/g2.log 2>&1 || { tail -20 gpurun_out/parity/g2.log; exit 1; }
loss gpurun_out/parity/g2.log gpt2_pp2
