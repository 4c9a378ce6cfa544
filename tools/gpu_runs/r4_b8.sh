#!/bin/bash
# 16-bit-uniform dropout layout: kernel + pipeline tests, epilogue probe; same-box A/B r3 / 977d2cb / HEAD;
# Pipe vs engine under rocprofv3.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "linear or gemm or dropout or gelu or act or bias or feedforward or embedding" > gpurun_out/b8_tests.log 2>&1 || { tail -40 gpurun_out/b8_tests.log; exit 1; }
tail -1 gpurun_out/b8_tests.log
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pipeline.py tests/test_gpu_fp32.py \
  -k "recompute or dropout or bit or fp32 or checkpoint" > gpurun_out/b8_tests2.log 2>&1 || { tail -40 gpurun_out/b8_tests2.log; exit 1; }
tail -1 gpurun_out/b8_tests2.log
timeout -k 10 200 python -u tools/epilogue_cost_probe.py > gpurun_out/epilogue_probe8.txt 2>&1; cat gpurun_out/epilogue_probe8.txt
bash tools/gpu_runs/r4_b7.sh
