#!/bin/bash
# Round 6: hipMemcpyDeviceToDeviceNoCU through torch's bundled HIP runtime: accepted?  DMA or kernel?
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/nocu_torch -o nt -- python3 tools/nocu_torch_probe.py > gpurun_out/nocu_torch.log 2>&1 || { tail -20 gpurun_out/nocu_torch.log; exit 1; }
grep -v "^W20\|rocprofv3" gpurun_out/nocu_torch.log | tail -8
python - <<'PY'
import glob, sqlite3
db = glob.glob("gpurun_out/nocu_torch/**/*.db", recursive=True)[0]
c = sqlite3.connect(db)
print("copy kernels:", c.execute("select grid_x, count(*) from kernels where name like '%copyBuffer%' group by grid_x").fetchall())
print("DMA copies:", c.execute("select size, count(*), name from memory_copies group by size, name").fetchall())
PY
