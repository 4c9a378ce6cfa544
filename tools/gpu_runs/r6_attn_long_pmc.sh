#!/bin/bash
# Where the GPT-2-XL long-sequence attention kernels spend their cycles (B=16 S=1024 H=25 D=64 causal p=0.1).
set -o pipefail
mkdir -p gpurun_out/attn_long
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A="16 1024 25 64 causal 0.1"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU --kernel-trace -d gpurun_out/attn_long/a -o run -- python3 tools/bench_attn.py $A > gpurun_out/attn_long/a.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS --kernel-trace -d gpurun_out/attn_long/b -o run -- python3 tools/bench_attn.py $A > gpurun_out/attn_long/b.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/attn_long/c -o run -- python3 tools/bench_attn.py $A > gpurun_out/attn_long/c.log 2>&1
rc=$?
for d in a b c; do f=$(find gpurun_out/attn_long/$d -name "*.db" | head -1); [ -n "$f" ] && python3 tools/pmc_db.py $f attn_long > gpurun_out/attn_long/$d.txt 2>&1; python3 tools/kstats_db.py $f > gpurun_out/attn_long/$d.k.txt 2>&1; done
find gpurun_out/attn_long -name "*.db" -delete
tail -3 gpurun_out/attn_long/*.log
exit $rc
