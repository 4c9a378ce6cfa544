#!/bin/bash
# Round 5: Adam under three chip states (power probe), then the PP=8 plan tables with the emulated pick.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 MIPIPE_CALIB_DIR="$GRAFT_REPO_ROOT/gpurun_out/calib"
timeout -k 10 240 python -u tools/adam_power_probe.py > gpurun_out/adam_power.txt 2>&1 || { tail -20 gpurun_out/adam_power.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/adam_power.txt
bash tools/gpu_runs/r5_g16.sh enc12_d4096:8:330 gpt2_xl:8:540
