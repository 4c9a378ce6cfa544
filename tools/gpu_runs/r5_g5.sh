#!/bin/bash
# Round 5: transport 'auto' GPU tests (+ the IPC link tests), then the 2-rank shared-GPU rehearsal at real enc12
# shapes (6 layers per rank, micro-batch 64, chunks 8) with the inline and the copy-stream (sdma) engines, profiled.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 GPU_MAX_HW_QUEUES=16
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pipeline.py -k "ipc or auto" > gpurun_out/r5_ipc_tests.log 2>&1 || { tail -40 gpurun_out/r5_ipc_tests.log; exit 1; }
tail -3 gpurun_out/r5_ipc_tests.log
for eng in inline sdma; do
  MIPIPE_IPC_ENGINE=$eng timeout -k 10 500 python -u tools/profile_ranks.py --nproc 2 --out gpurun_out/tl_$eng -- --shared-gpu --config enc12_d4096 --micro-batch 64 --chunks 8 --steps 2 --warmup 1 --no-bubble > gpurun_out/tl_$eng.txt 2>&1 || { tail -30 gpurun_out/tl_$eng.txt; exit 1; }
  echo "== engine $eng"; grep -v "^\[" gpurun_out/tl_$eng.txt | tail -8
  rm -rf gpurun_out/tl_$eng
done
