#!/bin/bash
# Round 5: same-box GEMM main-loop comparison -- the 4-wave harness schedules vs the product 8-wave / 4-wave K sweeps.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
for w in 8 4; do
  MIPIPE_GEMM_WAVES=$w timeout -k 10 200 python -u tools/gemm_k_sweep.py 8192 4096 > gpurun_out/ksweep6_w$w.txt 2>&1 || { tail gpurun_out/ksweep6_w$w.txt; exit 1; }
  echo "product waves $w:"; tail -4 gpurun_out/ksweep6_w$w.txt
done
timeout -k 10 180 tools/micro/bin/gemm4w 8192 4096 > gpurun_out/gemm4w_sched6.txt 2>&1 || { cat gpurun_out/gemm4w_sched6.txt; exit 1; }
tail -14 gpurun_out/gemm4w_sched6.txt
MIPIPE_GEMM_WAVES=8 timeout -k 10 200 python -u tools/gemm_k_sweep.py 8192 4096 > gpurun_out/ksweep6b_w8.txt 2>&1 || { tail gpurun_out/ksweep6b_w8.txt; exit 1; }
echo "product waves 8 again:"; tail -4 gpurun_out/ksweep6b_w8.txt
