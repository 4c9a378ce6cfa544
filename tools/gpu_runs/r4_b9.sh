#!/bin/bash
# Multi-round GEMM grids: one launch (MIPIPE_GEMM_ROUNDS=0) vs one launch per round of tiles (default), same box.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
val() { grep -o '"value": [0-9.]*' "$1" | head -1; }
for i in 1 2; do
  for r in 1 0; do
    MIPIPE_GEMM_ROUNDS=$r timeout -k 10 300 python -u bench.py --config gpt2_xl --steps 4 --warmup 2 --no-bubble > gpurun_out/b9_gpt_r${r}_$i.log 2>&1 || { tail -20 gpurun_out/b9_gpt_r${r}_$i.log; exit 1; }
    echo "gpt2_xl rounds=$r run $i: $(val gpurun_out/b9_gpt_r${r}_$i.log)"
  done
done
for i in 1 2; do
  for r in 1 0; do
    MIPIPE_GEMM_ROUNDS=$r timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-bubble > gpurun_out/b9_enc_r${r}_$i.log 2>&1 || { tail -20 gpurun_out/b9_enc_r${r}_$i.log; exit 1; }
    echo "enc12 rounds=$r run $i: $(val gpurun_out/b9_enc_r${r}_$i.log)"
  done
done
bash tools/gpu_runs/r4_pmc_attn.sh || exit 1
for d in pmca1 pmca2; do python3 tools/pmc_db.py gpurun_out/$d/*.db attn 2>&1 | head -40; done
