#!/bin/bash
# Round 5, VERDICT r4 item 5: every PP=8 plan alternative emulated rank by rank (tools/plan_table.py).
# usage: r5_g12.sh <config>
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 MIPIPE_CALIB_DIR="$GRAFT_REPO_ROOT/gpurun_out/calib"
timeout -k 10 1080 python -u tools/plan_table.py --config "$1" --v 1,2,3,4 --steps 4 > gpurun_out/plan_table_$1.txt 2>&1 || { tail -30 gpurun_out/plan_table_$1.txt; exit 1; }
grep -v "^wall\|^# PP=8 rank" gpurun_out/plan_table_$1.txt | tail -25
