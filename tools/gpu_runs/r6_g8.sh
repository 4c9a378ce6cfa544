#!/bin/bash
# Round 6: epilogue operand prefetch (dgrad residual / activation-mask reads, forward residual reads) -- GEMM kernel
# tests, then the bench, the roofline profile (dgrad vs forward of the same shape), GPT-2-XL.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "gemm or linear" -p no:cacheprovider > gpurun_out/g8_tests.log 2>&1 || { tail -30 gpurun_out/g8_tests.log; exit 1; }
tail -1 gpurun_out/g8_tests.log
bash tools/gpu_runs/r6_prof.sh
