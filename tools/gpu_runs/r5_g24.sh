#!/bin/bash
# Round 5: NoCU copies (copy engines only) -- probe under rocprofv3 (which copy launches a kernel), then the IPC /
# transport-auto GPU tests with the slot-reuse self-test and the NoCU sdma engine, then the sdma rehearsal at enc12.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 GPU_MAX_HW_QUEUES=16
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_nocu -o run -- ./tools/micro/bin/nocu_copy > gpurun_out/nocu_copy.txt 2>&1 || { tail -20 gpurun_out/nocu_copy.txt; exit 1; }
grep -v "^W2\|^E2\|rocprofv3\|amdgpu.ids" gpurun_out/nocu_copy.txt | head -12
python3 tools/prof_summary.py gpurun_out/prof_nocu/run_results.db 10 > gpurun_out/nocu_kernels.txt 2>&1; cat gpurun_out/nocu_kernels.txt
rm -rf gpurun_out/prof_nocu
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pipeline.py -k "ipc or auto" > gpurun_out/r5_ipc_tests2.log 2>&1 || { tail -40 gpurun_out/r5_ipc_tests2.log; exit 1; }
tail -3 gpurun_out/r5_ipc_tests2.log
MIPIPE_IPC_ENGINE=sdma timeout -k 10 500 python -u tools/profile_ranks.py --nproc 2 --out gpurun_out/tln_sdma -- --shared-gpu --config enc12_d4096 --micro-batch 64 --chunks 8 --steps 2 --warmup 1 --no-bubble > gpurun_out/tln_sdma.txt 2>&1 || { tail -30 gpurun_out/tln_sdma.txt; exit 1; }
echo "== engine sdma (NoCU)"; grep -v "^\[" gpurun_out/tln_sdma.txt | tail -6
rm -rf gpurun_out/tln_sdma
