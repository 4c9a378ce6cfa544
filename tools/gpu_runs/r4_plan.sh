#!/bin/bash
# Measured-cost planning: PP=8 rank emulation of configs #3 (enc12 except_last) and #4 (GPT-2-XL always), analytic vs measured.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 MIPIPE_CALIB_DIR=$GRAFT_REPO_ROOT/gpurun_out/calib
for cfg in gpt2_xl enc12_d4096; do
  for plan in analytic measured; do
    timeout -k 10 500 python -u tools/pp_rank_emulation.py --config $cfg --ranks all --steps 4 --plan $plan > gpurun_out/emu_${cfg}_${plan}.log 2>&1 || { tail -20 gpurun_out/emu_${cfg}_${plan}.log; exit 1; }
    grep "^#\|^wall" gpurun_out/emu_${cfg}_${plan}.log | grep -v "^# PP=" | tail -14
  done
done
