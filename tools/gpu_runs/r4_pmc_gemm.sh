#!/bin/bash
# Round-4 GEMM PMC passes (one counter set per run, kernel-trace only) over the 4096^3 layout ablation: forward
# <A_KC,B_KC>, dgrad / transposed weight gradient <A_KC,!B_KC>, both-I-contiguous weight gradient <!A_KC,!B_KC>.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE --kernel-trace -d gpurun_out/pmc4a -o p1 -- python3 tools/gemm_ablate.py 4096 > gpurun_out/pmc4a.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d gpurun_out/pmc4b -o p2 -- python3 tools/gemm_ablate.py 4096 > gpurun_out/pmc4b.log 2>&1

for d in pmc4a pmc4b; do python3 tools/pmc_db.py gpurun_out/$d/*.db gemm256 > gpurun_out/$d.txt 2>&1; done
cat gpurun_out/pmc4a.txt gpurun_out/pmc4b.txt | head -120
rm -rf gpurun_out/pmc4a gpurun_out/pmc4b
