#!/bin/bash
# Round 5: overlapped Adam (FlatAdam(overlap_modules=...)): numerics, then a same-box A/B with the driver's command.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 120 python -c "import torch; print('stream priority range', torch.cuda.Stream.priority_range())"
timeout -k 10 300 python -u -m pytest tests/test_gpu_optim_overlap.py -v --timeout 120 --timeout-method thread > gpurun_out/r5_overlap_tests.log 2>&1 || { tail -40 gpurun_out/r5_overlap_tests.log; exit 1; }
tail -2 gpurun_out/r5_overlap_tests.log
for arm in off on on off on off; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --opt-overlap $arm > gpurun_out/ov_$arm.log 2>&1 || { tail -20 gpurun_out/ov_$arm.log; exit 1; }
  echo "opt-overlap $arm: $(grep -o '"value": [0-9.]*' gpurun_out/ov_$arm.log) $(grep -o '"gfxclk_mhz": {[^}]*}' gpurun_out/ov_$arm.log) $(grep -o '"power_limited_pct": [0-9.]*' gpurun_out/ov_$arm.log)"
done
for arm in off on; do
  timeout -k 10 300 python -u bench.py --config gpt2_xl --steps 10 --warmup 3 --no-bubble --opt-overlap $arm > gpurun_out/ovg_$arm.log 2>&1 || { tail -20 gpurun_out/ovg_$arm.log; exit 1; }
  echo "gpt2_xl opt-overlap $arm: $(grep -o '"value": [0-9.]*' gpurun_out/ovg_$arm.log)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ov -o run -- python3 bench.py --steps 4 --warmup 2 --no-bubble --opt-overlap on > gpurun_out/prof_ov.log 2>&1 || { tail -5 gpurun_out/prof_ov.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof_ov/run_results.db 30 --by-grid > gpurun_out/prof_ov.txt 2>&1
python3 tools/overlap_share.py gpurun_out/prof_ov/run_results.db adam >> gpurun_out/prof_ov.txt 2>&1
tail -2 gpurun_out/prof_ov.txt
rm -rf gpurun_out/prof_ov
head -20 gpurun_out/prof_ov.txt
# GPT-2-XL PP=8: the default plan vs the best alternative, 3 alternating repeats (noise of the plan table)
export MIPIPE_CALIB_DIR="$GRAFT_REPO_ROOT/gpurun_out/calib"
timeout -k 10 420 python -u tools/plan_table.py --config gpt2_xl --labels DEFAULT,analytic/makespan/v=4 --repeats 3 > gpurun_out/plan_repeat_gpt2_xl.txt 2>&1 || { tail -30 gpurun_out/plan_repeat_gpt2_xl.txt; exit 1; }
grep "^   walls\|^## plan" gpurun_out/plan_repeat_gpt2_xl.txt | cut -c1-200
