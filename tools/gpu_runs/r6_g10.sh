#!/bin/bash
# Round 6: the ReLU (+ dropout) mask handed to fc2's folded dgrad as bits (kActReluBits) -- kernel tests, then the
# driver's bench command with and without (MIPIPE_RELU_BITS=0), arms interleaved, and the dgrad split.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "gemm or linear or fold or relu" -p no:cacheprovider > gpurun_out/g10_tests.log 2>&1 || { tail -30 gpurun_out/g10_tests.log; exit 1; }
tail -1 gpurun_out/g10_tests.log
for i in 1 2; do
  for b in 0 1; do
    MIPIPE_RELU_BITS=$b timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/g10_b${b}_$i.log 2>&1 || { tail -20 gpurun_out/g10_b${b}_$i.log; exit 1; }
    echo "bits=$b run $i: $(grep -o '"value": [0-9.]*' gpurun_out/g10_b${b}_$i.log) $(grep -o '"gfxclk_mhz": {"mean": [0-9.]*' gpurun_out/g10_b${b}_$i.log)"
  done
done
bash tools/gpu_runs/r6_g9.sh
