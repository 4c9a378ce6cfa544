#!/bin/bash
# Round 5: 4-wave GEMM product A/B (numerics + per-shape timing), then the enc12 / GPT-2-XL step with 8 vs 4 waves.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/gemm_waves_ab.py 8192 > gpurun_out/gemm_waves_ab.txt 2>&1 || { cat gpurun_out/gemm_waves_ab.txt; exit 1; }
cat gpurun_out/gemm_waves_ab.txt
for rep in 1 2; do
  for w in 8 4; do
    MIPIPE_GEMM_WAVES=$w timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/ab_enc_w${w}_$rep.log 2>&1 || { tail -20 gpurun_out/ab_enc_w${w}_$rep.log; exit 1; }
    echo "enc12 waves=$w rep=$rep: $(grep -o '"value": [0-9.]*' gpurun_out/ab_enc_w${w}_$rep.log) $(grep -o '"gfxclk_mhz": {[^}]*}' gpurun_out/ab_enc_w${w}_$rep.log)"
  done
done
for w in 8 4; do
  MIPIPE_GEMM_WAVES=$w timeout -k 10 300 python -u bench.py --config gpt2_xl --steps 10 --warmup 3 --no-bubble > gpurun_out/ab_gpt_w${w}.log 2>&1 || { tail -20 gpurun_out/ab_gpt_w${w}.log; exit 1; }
  echo "gpt2_xl waves=$w: $(grep -o '"value": [0-9.]*' gpurun_out/ab_gpt_w${w}.log)"
done
