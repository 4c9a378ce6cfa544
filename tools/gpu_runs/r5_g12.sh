#!/bin/bash
# Round 5, VERDICT r4 item 5: every PP=8 plan alternative emulated rank by rank (tools/plan_table.py).
# usage: r5_g12.sh <config>:<seconds> ...
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 MIPIPE_CALIB_DIR="$GRAFT_REPO_ROOT/gpurun_out/calib"
for spec in "$@"; do
  c=${spec%%:*}; t=${spec##*:}
  timeout -k 10 $t python -u tools/plan_table.py --config "$c" --v 1,2,3,4 --steps 4 > gpurun_out/plan_table_$c.txt 2>&1 || { tail -30 gpurun_out/plan_table_$c.txt; exit 1; }
  grep -v "^wall\|^# PP=8 rank\|^## plan\|^   walls" gpurun_out/plan_table_$c.txt | tail -20
done
