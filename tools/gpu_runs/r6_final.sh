#!/bin/bash
# Round 6 state: the GPU tier, smoke, the driver's bench command (twice), GPT-2-XL (config #4 shape, 20 steps after 5 warm-up).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/final_gpu_r6.log 2>&1
rc=$?
tail -3 gpurun_out/final_gpu_r6.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^ERROR" gpurun_out/final_gpu_r6.log | head; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke_r6.log 2>&1 || { tail -10 gpurun_out/final_smoke_r6.log; exit 1; }
tail -1 gpurun_out/final_smoke_r6.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final_bench_r6_$i.log 2>&1 || { tail -20 gpurun_out/final_bench_r6_$i.log; exit 1; }
  echo "bench $i: $(grep -o '"value": [0-9.]*' gpurun_out/final_bench_r6_$i.log) $(grep -o '"gfxclk_mhz": {[^}]*}' gpurun_out/final_bench_r6_$i.log) $(grep -o '"power_limited_pct": [0-9.]*' gpurun_out/final_bench_r6_$i.log)"
done
timeout -k 10 400 python -u bench.py --config gpt2_xl --steps 20 --warmup 5 --no-bubble > gpurun_out/final_gpt_r6.log 2>&1 || { tail -20 gpurun_out/final_gpt_r6.log; exit 1; }
echo "gpt2_xl: $(grep -o '"value": [0-9.]*' gpurun_out/final_gpt_r6.log) $(grep -o '"gfxclk_mhz": {[^}]*}' gpurun_out/final_gpt_r6.log)"
