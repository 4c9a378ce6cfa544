#!/bin/bash
# Round 6: the CU-free IPC links (DMA payload + DMA flag copy on the copy stream, host-polled release counter):
# IPC / auto GPU tests, then the 2-rank shared-GPU enc12 rehearsal for both engines, profiled (kernel + marker
# traces); engine_timeline now excludes the stream-op spin kernels from busy.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 GPU_MAX_HW_QUEUES=16
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_pipeline.py -k "ipc or auto" > gpurun_out/r6_ipc_tests.log 2>&1 || { tail -60 gpurun_out/r6_ipc_tests.log; exit 1; }
tail -3 gpurun_out/r6_ipc_tests.log
for eng in sdma inline; do
  MIPIPE_IPC_ENGINE=$eng timeout -k 10 400 python -u tools/profile_ranks.py --nproc 2 --copy-trace --out gpurun_out/tl6_$eng -- --shared-gpu --config enc12_d4096 --micro-batch 64 --chunks 8 --steps 2 --warmup 1 --no-bubble > gpurun_out/tl6_$eng.txt 2>&1 || { tail -30 gpurun_out/tl6_$eng.txt; exit 1; }
  echo "== engine $eng"; grep -v "^\[" gpurun_out/tl6_$eng.txt | tail -8
done
