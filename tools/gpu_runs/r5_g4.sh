#!/bin/bash
# Round 5: CU-hold probe (+ driver-exact bench with telemetry, hipBLASLt kernel id), then same-box K sweeps of the
# 8-wave and 4-wave product GEMMs.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
bash tools/gpu_runs/r5_hold.sh || exit $?
for w in 8 4; do
  MIPIPE_GEMM_WAVES=$w timeout -k 10 200 python -u tools/gemm_k_sweep.py 8192 4096 > gpurun_out/ksweep_w$w.txt 2>&1 || { tail gpurun_out/ksweep_w$w.txt; exit 1; }
  echo "waves $w:"; tail -9 gpurun_out/ksweep_w$w.txt
done
