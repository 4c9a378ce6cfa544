#!/bin/bash
# SQ counters of the long-sequence dK/dV kernels, 4-wave (MIPIPE_ATTN_DKDV8=0) vs 8-wave (=1), GPT-2-XL shape.
set -o pipefail
mkdir -p gpurun_out/dkdv8_pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for arm in 0 1; do
  timeout -s KILL 90 env MIPIPE_ATTN_DKDV8=$arm rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA --kernel-trace -d gpurun_out/dkdv8_pmc/a$arm -o run -- python3 tools/bench_attn.py 18 1024 25 64 causal 0.1 > gpurun_out/dkdv8_pmc/a$arm.log 2>&1 || exit 1
  python3 tools/pmc_db.py $(find gpurun_out/dkdv8_pmc/a$arm -name "*.db" | head -1) dkdv > gpurun_out/dkdv8_pmc/a$arm.txt 2>&1
  python3 tools/kstats_db.py $(find gpurun_out/dkdv8_pmc/a$arm -name "*.db" | head -1) dkdv >> gpurun_out/dkdv8_pmc/a$arm.txt 2>&1
done
find gpurun_out/dkdv8_pmc -name "*.db" -delete
cat gpurun_out/dkdv8_pmc/a0.txt gpurun_out/dkdv8_pmc/a1.txt
