#!/bin/bash
# GPT-2-XL weight-gradient GEMMs (19 % of the step at ~1.0 PF/s): block width 128 vs auto; x^T for every weight.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
val() { grep -o '"value": [0-9.]*' "$1" | head -1; }
for i in 1 2; do
  for arm in base w128 xtall; do
    envs=""
    [ $arm = w128 ] && envs="MIPIPE_GEMM_W=128"
    [ $arm = xtall ] && envs="MIPIPE_WGRAD_XT_MIN_N=0 MIPIPE_WGRAD_XT_MIN_TILES=0"
    env $envs timeout -k 10 300 python -u bench.py --config gpt2_xl --steps 4 --warmup 2 --no-bubble > gpurun_out/b14_${arm}_$i.log 2>&1 || { tail -20 gpurun_out/b14_${arm}_$i.log; exit 1; }
    echo "gpt2_xl $arm run $i: $(val gpurun_out/b14_${arm}_$i.log)"
  done
done
