#!/bin/bash
# GPT-2-XL (config #4) at PP=1: GELU'(pre) saved + folded, flush-time x^T, bias fold -- A/B and a kernel profile.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
val() { grep -o '"value": [0-9.]*' "$1" | head -1; }
for i in 1 2; do
  for arm in "new" "old"; do
    if [ $arm = old ]; then envs="MIPIPE_GELU_SAVE_GRAD=0 MIPIPE_WGRAD_XT=0"; else envs=""; fi
    env $envs timeout -k 10 300 python -u bench.py --config gpt2_xl --steps 4 --warmup 2 --no-bubble > gpurun_out/gpt_${arm}_$i.log 2>&1 || { tail -20 gpurun_out/gpt_${arm}_$i.log; exit 1; }
    echo "gpt2_xl $arm run $i: $(val gpurun_out/gpt_${arm}_$i.log) $(grep -o '"peak_hbm_gib_per_gpu": \[[0-9., ]*\]' gpurun_out/gpt_${arm}_$i.log)"
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gpt4 -o run -- python3 bench.py --config gpt2_xl --steps 2 --warmup 1 --no-bubble > gpurun_out/prof_gpt4.log 2>&1 || { tail -5 gpurun_out/prof_gpt4.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof_gpt4/run_results.db 30 2>&1 | head -34
