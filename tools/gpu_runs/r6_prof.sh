#!/bin/bash
# Round 6 step profiles: enc12 PP=1 (bench defaults) with the per-GEMM-class roofline at the step's gfxclk, and
# GPT-2-XL.  The clock comes from an unprofiled bench run's JSON telemetry right before.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6p_bench.log 2>&1 || { tail -20 gpurun_out/r6p_bench.log; exit 1; }
clk=$(python -c "import json; d=[json.loads(l) for l in open('gpurun_out/r6p_bench.log') if l.startswith('{')][0]; print(d['telemetry']['gfxclk_mhz']['mean'])")
echo "bench: $(grep -o '"value": [0-9.]*' gpurun_out/r6p_bench.log) gfxclk mean $clk"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r6e -o run -- python3 bench.py --steps 4 --warmup 2 --no-bubble > gpurun_out/prof_r6e.log 2>&1 || { tail -5 gpurun_out/prof_r6e.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof_r6e/run_results.db 30 --by-grid > gpurun_out/prof_r6e.txt 2>&1
python3 tools/gemm_roofline.py gpurun_out/prof_r6e/run_results.db --steps 6 --gfxclk $clk > gpurun_out/roofline_r6e.txt 2>&1
python3 tools/gemm_roofline.py gpurun_out/prof_r6e/run_results.db --steps 6 --gfxclk 1800 | tail -1 >> gpurun_out/roofline_r6e.txt 2>&1
echo "enc12 profiled: $(grep -o '"value": [0-9.]*' gpurun_out/prof_r6e.log)"; cat gpurun_out/roofline_r6e.txt
rm -rf gpurun_out/prof_r6e
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r6g -o run -- python3 bench.py --config gpt2_xl --steps 2 --warmup 1 --no-bubble > gpurun_out/prof_r6g.log 2>&1 || { tail -5 gpurun_out/prof_r6g.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof_r6g/run_results.db 30 > gpurun_out/prof_r6g.txt 2>&1
echo "gpt2_xl profiled: $(grep -o '"value": [0-9.]*' gpurun_out/prof_r6g.log)"; head -3 gpurun_out/prof_r6g.txt
rm -rf gpurun_out/prof_r6g
