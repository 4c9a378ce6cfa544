#!/bin/bash
# Round 5 final kernel profiles: enc12 PP=1 at the new default micro-batch 128, and GPT-2-XL.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5e -o run -- python3 bench.py --steps 4 --warmup 2 --no-bubble > gpurun_out/prof_r5e.log 2>&1 || { tail -5 gpurun_out/prof_r5e.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof_r5e/run_results.db 30 --by-grid > gpurun_out/prof_r5e.txt 2>&1
echo "enc12 profiled: $(grep -o '"value": [0-9.]*' gpurun_out/prof_r5e.log)"; head -3 gpurun_out/prof_r5e.txt
rm -rf gpurun_out/prof_r5e
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5g -o run -- python3 bench.py --config gpt2_xl --steps 2 --warmup 1 --no-bubble > gpurun_out/prof_r5g.log 2>&1 || { tail -5 gpurun_out/prof_r5g.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof_r5g/run_results.db 30 > gpurun_out/prof_r5g.txt 2>&1
echo "gpt2_xl profiled: $(grep -o '"value": [0-9.]*' gpurun_out/prof_r5g.log)"; head -3 gpurun_out/prof_r5g.txt
rm -rf gpurun_out/prof_r5g
