#!/bin/bash
# Round 5: overlapped-Adam tests (embedding atomics tolerated); plan tables for the bench's enc12 PP=2 / PP=4 defaults.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 MIPIPE_CALIB_DIR="$GRAFT_REPO_ROOT/gpurun_out/calib"
timeout -k 10 300 python -u -m pytest tests/test_gpu_optim_overlap.py -v --timeout 120 --timeout-method thread > gpurun_out/r5_overlap_tests.log 2>&1 || { tail -40 gpurun_out/r5_overlap_tests.log; exit 1; }
tail -2 gpurun_out/r5_overlap_tests.log
for pp in 2 4; do
  timeout -k 10 480 python -u tools/plan_table.py --config enc12_d4096 --pp $pp --v 1,2,3,4 --steps 4 > gpurun_out/plan_table_enc12_pp$pp.txt 2>&1 || { tail -30 gpurun_out/plan_table_enc12_pp$pp.txt; exit 1; }
  grep -v "^wall\|^# PP=\|^## plan\|^   walls" gpurun_out/plan_table_enc12_pp$pp.txt | tail -18
done
