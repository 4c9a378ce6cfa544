#!/bin/bash
# HBM bytes and stall counters of the S = 128 attention kernels, one run per counter set.
set -o pipefail
mkdir -p gpurun_out/attn_pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/attn_pmc/f -o run -- python3 tools/bench_attn.py > gpurun_out/attn_pmc/f.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/attn_pmc/w -o run -- python3 tools/bench_attn.py > gpurun_out/attn_pmc/w.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_WAIT_INST_ANY --kernel-trace -d gpurun_out/attn_pmc/s -o run -- python3 tools/bench_attn.py > gpurun_out/attn_pmc/s.log 2>&1
rc=$?
echo "rc=$rc"
for d in f w s; do python3 tools/pmc_db.py $(find gpurun_out/attn_pmc/$d -name "*.db" | head -1) s128 > gpurun_out/attn_pmc/$d.txt 2>&1; done
find gpurun_out/attn_pmc -name "*.db" -delete
exit $rc
