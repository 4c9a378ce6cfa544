#!/bin/bash
# Round 6: which copies does the runtime run as kernels?  small_copy_probe under a kernel + memory-copy trace, with
# the default settings and with GPU_FORCE_BLIT_COPY_SIZE=0.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/scp_def -o scp -- tools/micro/bin/small_copy_probe > gpurun_out/scp_def.log 2>&1 || { tail -20 gpurun_out/scp_def.log; exit 1; }
python tools/small_copy_report.py "gpurun_out/scp_def/**/*.db"
export GPU_FORCE_BLIT_COPY_SIZE=0
timeout -k 10 60 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/scp_f0 -o scp -- tools/micro/bin/small_copy_probe > gpurun_out/scp_f0.log 2>&1 || { tail -20 gpurun_out/scp_f0.log; exit 1; }
echo "== GPU_FORCE_BLIT_COPY_SIZE=0"
python tools/small_copy_report.py "gpurun_out/scp_f0/**/*.db"
