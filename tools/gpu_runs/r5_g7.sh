#!/bin/bash
# Round 5: Pipe after the shared-stream fix (ref_main fp32, balance 8,8) + the Pipe transport tests; then the 4-wave
# GEMM A/B after the row-split epilogue / schedule 2 (K sweeps + shapes).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
for ck in never except_last; do
  timeout -k 10 300 python -u bench.py --impl pipe --pipe-balance 8,8 --config ref_main --dtype fp32 --checkpoint $ck --steps 10 --warmup 3 > gpurun_out/pg2_$ck.log 2>&1 || { tail -20 gpurun_out/pg2_$ck.log; exit 1; }
  echo "pipe88 $ck (shared stage streams): $(grep -o '"value": [0-9.]*' gpurun_out/pg2_$ck.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/pg2_$ck.log)"
done
timeout -k 10 300 python -u bench.py --config ref_main --dtype fp32 --checkpoint except_last --chunks 4 --micro-batch 8 --steps 10 --warmup 3 --no-bubble > gpurun_out/pg2_engine_el.log 2>&1 || { tail -20 gpurun_out/pg2_engine_el.log; exit 1; }
echo "engine except_last: $(grep -o '"value": [0-9.]*' gpurun_out/pg2_engine_el.log)"
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pipe_transport.py > gpurun_out/pipe_transport_tests.log 2>&1 || { tail -30 gpurun_out/pipe_transport_tests.log; exit 1; }
tail -2 gpurun_out/pipe_transport_tests.log
for w in 8 4; do
  MIPIPE_GEMM_WAVES=$w timeout -k 10 200 python -u tools/gemm_k_sweep.py 8192 4096 > gpurun_out/ksweep7_w$w.txt 2>&1 || { tail gpurun_out/ksweep7_w$w.txt; exit 1; }
  echo "product waves $w:"; tail -4 gpurun_out/ksweep7_w$w.txt
done
timeout -k 10 300 python -u tools/gemm_waves_ab.py 8192 > gpurun_out/gemm_waves_ab3.txt 2>&1 || { cat gpurun_out/gemm_waves_ab3.txt; exit 1; }
cat gpurun_out/gemm_waves_ab3.txt
