#!/bin/bash
# Round 5: Adam default = streaming stores: kernel tests, three consecutive step profiles (Adam ms per step),
# driver-command bench; GEMM burst vs sustained clock probe.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -k "adam or sumsq" --timeout 120 --timeout-method thread > gpurun_out/r5_adam_tests.log 2>&1 || { tail -30 gpurun_out/r5_adam_tests.log; exit 1; }
tail -1 gpurun_out/r5_adam_tests.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5_bench2.log 2>&1 || { tail -20 gpurun_out/r5_bench2.log; exit 1; }
echo "bench: $(grep -o '"value": [0-9.]*' gpurun_out/r5_bench2.log) $(grep -o '"gfxclk_mhz": {[^}]*}' gpurun_out/r5_bench2.log)"
for i in 1 2 3; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_a$i -o run -- python3 bench.py --steps 4 --warmup 2 --no-bubble > gpurun_out/prof_a$i.log 2>&1 || { tail -5 gpurun_out/prof_a$i.log; exit 1; }
  python3 tools/prof_summary.py gpurun_out/prof_a$i/run_results.db 40 --by-grid > gpurun_out/prof_a$i.txt 2>&1
  echo "profile $i: $(grep -o '"value": [0-9.]*' gpurun_out/prof_a$i.log) | $(grep adam gpurun_out/prof_a$i.txt | cut -c1-60)"
  [ $i -eq 3 ] || rm -rf gpurun_out/prof_a$i
done
rm -rf gpurun_out/prof_a3
timeout -k 10 200 python -u tools/gemm_clock_probe.py > gpurun_out/gemm_clock.txt 2>&1 || { tail -20 gpurun_out/gemm_clock.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/gemm_clock.txt
