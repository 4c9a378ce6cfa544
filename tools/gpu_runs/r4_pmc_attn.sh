#!/bin/bash
# PMC passes over the GPT-2-XL attention (B 18, S 1024, H 25, D 64, causal, p 0.1): fwd / dK,dV / dQ kernels.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_VALU --kernel-trace -d gpurun_out/pmca1 -o p1 -- python3 tools/bench_attn.py 18 1024 25 64 causal 0.1 > gpurun_out/pmca1.log 2>&1 || { tail -5 gpurun_out/pmca1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES --kernel-trace -d gpurun_out/pmca2 -o p2 -- python3 tools/bench_attn.py 18 1024 25 64 causal 0.1 > gpurun_out/pmca2.log 2>&1 || { tail -5 gpurun_out/pmca2.log; exit 1; }
ls gpurun_out/pmca1 gpurun_out/pmca2
