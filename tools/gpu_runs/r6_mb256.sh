#!/bin/bash
# enc12 PP=1: micro-batch 256 x 128 vs the default 128 x 128 (chunks 4, never), the driver's command otherwise.
set -o pipefail
mkdir -p gpurun_out/mb
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
for i in 1 2; do
  for mb in 128 256; do
    timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --micro-batch $mb > gpurun_out/mb/b_${mb}_$i.log 2>&1 || { tail -20 gpurun_out/mb/b_${mb}_$i.log; exit 1; }
    echo "mb=$mb $i: $(grep -o '"value": [0-9.]*' gpurun_out/mb/b_${mb}_$i.log) $(grep -o '"gfxclk_mhz": {"mean": [0-9.]*' gpurun_out/mb/b_${mb}_$i.log) $(grep -o '"peak_hbm_gib_per_gpu": [^]]*]' gpurun_out/mb/b_${mb}_$i.log) $(grep -o '"power_limited_pct": [0-9.]*' gpurun_out/mb/b_${mb}_$i.log)"
  done
done
