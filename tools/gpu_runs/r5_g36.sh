#!/bin/bash
# Round 5: chunked IPC rings -- the ring sizes that stalled (2.0 / 3.0 GiB) now, the IPC GPU tests, and the PP=4
# shared-GPU rehearsal of the bench that stalled before.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 MIPIPE_IPC_DEBUG=1 GPU_MAX_HW_QUEUES=16
for spec in "64 32" "48 64"; do
  set -- $spec
  echo "== ring $1 x $2 MiB"
  timeout -k 10 60 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29681 tools/ipc_attach_probe.py 2 $1 $2 > gpurun_out/attach_chunked_$1_$2.txt 2>&1 || { echo "rc=$?"; grep -E "create|opening|mapped" gpurun_out/attach_chunked_$1_$2.txt | tail -4; exit 1; }
  grep -E "^rank|create" gpurun_out/attach_chunked_$1_$2.txt | head -4
done
unset MIPIPE_IPC_DEBUG
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pipeline.py -k "ipc or auto" > gpurun_out/r5_ipc_tests3.log 2>&1 || { tail -30 gpurun_out/r5_ipc_tests3.log; exit 1; }
tail -1 gpurun_out/r5_ipc_tests3.log
bash tools/gpu_runs/r5_g25.sh
