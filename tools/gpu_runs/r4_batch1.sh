#!/bin/bash
# Round 4, first batch: IPC signalling probe, GEMM race screen, x^T GEMM tests, same-box bench A/B of the
# x^T weight-gradient path, and the Pipe API numbers (engine vs --impl pipe, the reference's 2-partition
# structure on one GPU).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gemm_round_screen.py 30 > gpurun_out/round_screen.txt 2>&1 || { cat gpurun_out/round_screen.txt; exit 1; }
grep -c "all identical" gpurun_out/round_screen.txt; grep -v "all identical" gpurun_out/round_screen.txt | head -5
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "gemm or wgrad or linear or cross_entropy or x_transposed" > gpurun_out/xt_tests.log 2>&1 || { tail -40 gpurun_out/xt_tests.log; exit 1; }
tail -2 gpurun_out/xt_tests.log
val() { grep -o '"value": [0-9.]*' "$1" | head -1; }
for i in 1 2; do
  for xt in 0 1; do
    MIPIPE_WGRAD_XT=$xt timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-bubble > gpurun_out/xt_bench${xt}_$i.log 2>&1 || { tail -20 gpurun_out/xt_bench${xt}_$i.log; exit 1; }
    echo "enc12 xt=$xt run $i: $(val gpurun_out/xt_bench${xt}_$i.log) $(grep -o '"peak_hbm_gib_per_gpu": \[[0-9., ]*\]' gpurun_out/xt_bench${xt}_$i.log)"
  done
done
timeout -k 10 200 python -u bench.py --impl pipe --steps 10 --warmup 3 > gpurun_out/pipe_bench.log 2>&1 || { tail -20 gpurun_out/pipe_bench.log; exit 1; }
echo "enc12 --impl pipe: $(val gpurun_out/pipe_bench.log)"
for ck in never except_last; do
  timeout -k 10 200 python -u bench.py --impl pipe --config ref_main --dtype fp32 --pipe-balance 8,8 --checkpoint $ck --steps 10 --warmup 3 > gpurun_out/refmain_pipe2_$ck.log 2>&1 || { tail -20 gpurun_out/refmain_pipe2_$ck.log; exit 1; }
  echo "ref_main fp32 Pipe 2 partitions on one GPU, $ck: $(val gpurun_out/refmain_pipe2_$ck.log) $(grep -o '"peak_hbm_gib_per_gpu": \[[0-9., ]*\]' gpurun_out/refmain_pipe2_$ck.log)"
done
