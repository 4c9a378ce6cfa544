#!/bin/bash
# The bench's PP=8 plan pick and its refinement from measured walls, every rank emulated on one MI355X.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 MIPIPE_CALIB_DIR="$GRAFT_REPO_ROOT/gpurun_out/calib_refine"
timeout -k 10 900 python -u tools/plan_refine_probe.py --config enc12_d4096 --pp 8 --rounds 8 --refine-all --replan > gpurun_out/refine_pp8.log 2>&1
rc=$?
cat gpurun_out/refine_pp8.log | grep -v "^#.*rank\b" | tail -30
exit $rc
