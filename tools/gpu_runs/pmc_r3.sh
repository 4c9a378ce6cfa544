# PMC passes (one counter set per run, kernel-trace only) over the 4096^3 GEMM ablation on the default schedule 7
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE --kernel-trace -d gpurun_out/pmc1 -o p1 -- python3 tools/gemm_ablate.py 4096 > gpurun_out/pmc1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d gpurun_out/pmc2 -o p2 -- python3 tools/gemm_ablate.py 4096 > gpurun_out/pmc2.log 2>&1
