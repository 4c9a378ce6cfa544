#!/bin/bash
# Round-4 final state: the GPU tier, smoke, the default bench (enc12 PP=1), GPT-2-XL, and kernel profiles of both.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/final_gpu.log 2>&1
rc=$?
tail -4 gpurun_out/final_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || { tail -10 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/final_bench.log 2>&1 || { tail -20 gpurun_out/final_bench.log; exit 1; }
grep '"metric"' gpurun_out/final_bench.log | cut -c1-400
timeout -k 10 300 python -u bench.py --config gpt2_xl --steps 4 --warmup 2 --no-bubble > gpurun_out/final_gpt.log 2>&1 || { tail -20 gpurun_out/final_gpt.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/final_gpt.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final_enc -o run -- python3 bench.py --steps 4 --warmup 2 --no-bubble > gpurun_out/prof_final_enc.log 2>&1 || { tail -5 gpurun_out/prof_final_enc.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof_final_enc/run_results.db 30 --by-grid > gpurun_out/prof_final_enc.txt 2>&1
grep -o '"value": [0-9.]*' gpurun_out/prof_final_enc.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final_gpt -o run -- python3 bench.py --config gpt2_xl --steps 2 --warmup 1 --no-bubble > gpurun_out/prof_final_gpt.log 2>&1 || { tail -5 gpurun_out/prof_final_gpt.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof_final_gpt/run_results.db 30 > gpurun_out/prof_final_gpt.txt 2>&1
grep -o '"value": [0-9.]*' gpurun_out/prof_final_gpt.log
rm -rf gpurun_out/prof_final_enc gpurun_out/prof_final_gpt
