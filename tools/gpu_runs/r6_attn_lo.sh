#!/bin/bash
# S = 128 attention backward in 80 KiB (two workgroups per CU) vs 128 KiB: numerics, then timing.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu -k "attention_packed" > gpurun_out/attn_lo_tests.log 2>&1 || { tail -30 gpurun_out/attn_lo_tests.log; exit 1; }
tail -3 gpurun_out/attn_lo_tests.log
timeout -k 10 120 python -u tools/bench_attn.py 2>&1 | tee gpurun_out/attn_lo_bench.log
timeout -k 10 120 python -u tools/bench_attn.py 128 128 16 256 x 0.0 2>&1 | tee -a gpurun_out/attn_lo_bench.log
