#!/bin/bash
# Round 5: overlapped Adam -- where serial and overlapped differ, then the perf A/B regardless.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 120 python -c "import torch; print('stream priority range', torch.cuda.Stream.priority_range())"
timeout -k 10 300 python -u tools/overlap_debug.py 2>&1 | grep -v amdgpu.ids
sed -n '/^for arm in off on on off/,$p' tools/gpu_runs/r5_g13.sh > /tmp/rest.sh
bash /tmp/rest.sh
