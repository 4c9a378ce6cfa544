#!/bin/bash
# GPT-2-XL PP=2 (shared GPU) loss vs PP=1: the first step's loss (before any update), then 3 steps with the keep-word
# reuse off and with checkpoint='never', to place the difference.
set -o pipefail
mkdir -p gpurun_out/parity
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
loss() { python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print(sys.argv[2], 'loss', d['loss'], d['config']['parallelism'], d['config']['checkpoint'])" "$1" "$2"; }
p2() { local tag=$1; shift; timeout -k 10 400 env $ENVV python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29750 + RANDOM % 100)) bench.py --gpus 2 --shared-gpu "$@" > gpurun_out/parity/$tag.log 2>&1 || { tail -20 gpurun_out/parity/$tag.log; exit 1; }; loss gpurun_out/parity/$tag.log $tag; }
p1() { local tag=$1; shift; timeout -k 10 300 env $ENVV python -u bench.py "$@" > gpurun_out/parity/$tag.log 2>&1 || { tail -20 gpurun_out/parity/$tag.log; exit 1; }; loss gpurun_out/parity/$tag.log $tag; }
G="--config gpt2_xl --micro-batch 4 --chunks 8 --no-bubble"
ENVV="X=1"
p1 g1_first $G --steps 1 --warmup 0
p2 g2_first $G --steps 1 --warmup 0
ENVV="MIPIPE_ATTN_KEEP_REUSE=0"
p2 g2_noreuse $G --steps 3 --warmup 1
ENVV="X=1"
p2 g2_never $G --steps 3 --warmup 1 --checkpoint never
p1 g1_never $G --steps 3 --warmup 1 --checkpoint never
p2 g2_10 $G --steps 10 --warmup 1
