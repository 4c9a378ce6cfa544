#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/dm
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/dm -o run -- python3 tools/attn_long_dm_probe.py > gpurun_out/dm/log.txt 2>&1
rc=$?
python3 tools/kstats_db.py $(find gpurun_out/dm -name "*.db" | head -1) attn_long
find gpurun_out/dm -name "*.db" -delete
exit $rc
