#!/bin/bash
# Round 5: IPC self-test with the slot-reuse check -- the IPC / transport-auto GPU tests.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 GPU_MAX_HW_QUEUES=16
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pipeline.py -k "ipc or auto" > gpurun_out/r5_ipc_tests2.log 2>&1 || { tail -40 gpurun_out/r5_ipc_tests2.log; exit 1; }
tail -3 gpurun_out/r5_ipc_tests2.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --shared-gpu --transport auto --steps 3 --warmup 1 --no-bubble > gpurun_out/auto_shared.log 2>&1 || { tail -30 gpurun_out/auto_shared.log; exit 1; }
grep -o '"transport": "[^"]*"\|"value": [0-9.]*' gpurun_out/auto_shared.log
