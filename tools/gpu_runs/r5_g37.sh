#!/bin/bash
# Round 5: enc12 PP=1 micro-batch 128 (default) vs 192 vs 256, the driver's command, interleaved on one box.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
for mb in 128 192 256 128 192 256; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --micro-batch $mb > gpurun_out/mbb_$mb.log 2>&1 || { tail -20 gpurun_out/mbb_$mb.log; exit 1; }
  echo "mb $mb: $(grep -o '"value": [0-9.]*' gpurun_out/mbb_$mb.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/mbb_$mb.log) $(grep -o '"peak_hbm_gib_per_gpu": \[[^]]*\]' gpurun_out/mbb_$mb.log) $(grep -o '"gfxclk_mhz": {[^}]*}' gpurun_out/mbb_$mb.log)"
done
