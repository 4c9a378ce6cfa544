#!/bin/bash
# GPT-2-XL: flush-time x^T (transposed weight-gradient GEMM, bias folded) for the 1600-input weights too.
# Arms: default (x^T only for >= 6144 outputs and >= 512 tiles: none of GPT-2-XL's), fc1 (6400 outputs), qkv+fc1.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
val() { grep -o '"value": [0-9.]*' "$1" | head -1; }
for i in 1 2; do
  for arm in def fc1 qkvfc1; do
    envs="MIPIPE_WGRAD_XT_MIN_TILES=0"
    [ $arm = def ] && envs="MIPIPE_WGRAD_XT_MIN_TILES=512"
    [ $arm = qkvfc1 ] && envs="MIPIPE_WGRAD_XT_MIN_TILES=0 MIPIPE_WGRAD_XT_MIN_N=4800"
    env $envs timeout -k 10 300 python -u bench.py --config gpt2_xl --steps 4 --warmup 2 --no-bubble > gpurun_out/b20_${arm}_$i.log 2>&1 || { tail -20 gpurun_out/b20_${arm}_$i.log; exit 1; }
    echo "gpt2_xl $arm run $i: $(val gpurun_out/b20_${arm}_$i.log)"
  done
done
