#!/bin/bash
# Round 6: small NoCU copies into IPC-mapped memory -- DMA or kernel?  Default, ROC_P2P_SDMA_SIZE=0 / 1.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # $1 = tag
  rm -f /tmp/icp_h /tmp/icp_h.done
  timeout -k 10 90 tools/micro/bin/ipc_copy_probe export /tmp/icp_h > gpurun_out/icp_exp_$1.log 2>&1 &
  local exp=$!
  timeout -k 10 60 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/icp_$1 -o icp -- tools/micro/bin/ipc_copy_probe import /tmp/icp_h > gpurun_out/icp_$1.log 2>&1 || { tail -20 gpurun_out/icp_$1.log; kill $exp; return 1; }
  wait $exp || return 1
  python tools/small_copy_report.py "gpurun_out/icp_$1/**/*.db" --ipc
}
echo "== default"; run def || exit 1

