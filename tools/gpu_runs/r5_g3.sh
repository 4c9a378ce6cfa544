#!/bin/bash
# Round 5: harness schedules, then the product 4-wave kernel A/B (numerics + shapes + enc12 step).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 180 tools/micro/bin/gemm4w 8192 4096 > gpurun_out/gemm4w_sched.txt 2>&1 || { cat gpurun_out/gemm4w_sched.txt; exit 1; }
cat gpurun_out/gemm4w_sched.txt
timeout -k 10 300 python -u tools/gemm_waves_ab.py 8192 > gpurun_out/gemm_waves_ab2.txt 2>&1 || { cat gpurun_out/gemm_waves_ab2.txt; exit 1; }
cat gpurun_out/gemm_waves_ab2.txt
for rep in 1 2; do
  for w in 8 4; do
    MIPIPE_GEMM_WAVES=$w timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/ab2_enc_w${w}_$rep.log 2>&1 || { tail -20 gpurun_out/ab2_enc_w${w}_$rep.log; exit 1; }
    echo "enc12 waves=$w rep=$rep: $(grep -o '"value": [0-9.]*' gpurun_out/ab2_enc_w${w}_$rep.log) $(grep -o '"gfxclk_mhz": {[^}]*}' gpurun_out/ab2_enc_w${w}_$rep.log)"
  done
done
