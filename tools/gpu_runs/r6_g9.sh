#!/bin/bash
# Round 6: per-dgrad split of the enc12 step (which K=4096 dgrad is slower than the same-shape forward).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_g9 -o run -- python3 bench.py --steps 3 --warmup 1 --no-bubble > gpurun_out/prof_g9.log 2>&1 || { tail -5 gpurun_out/prof_g9.log; exit 1; }
python3 tools/dgrad_split.py gpurun_out/prof_g9/run_results.db
rm -rf gpurun_out/prof_g9
