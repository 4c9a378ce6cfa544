#!/bin/bash
# Attention images with the conflict-free swizzle: numerics, timing, bank-conflict counters.
set -o pipefail
mkdir -p gpurun_out/attn_swz
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu -k "attention" > gpurun_out/attn_swz/tests.log 2>&1 || { tail -30 gpurun_out/attn_swz/tests.log; exit 1; }
tail -2 gpurun_out/attn_swz/tests.log
timeout -k 10 120 python -u tools/bench_attn.py > gpurun_out/attn_swz/bench.log 2>&1 && \
timeout -k 10 120 python -u tools/bench_attn.py 128 128 16 256 x 0.0 >> gpurun_out/attn_swz/bench.log 2>&1 && \
timeout -k 10 120 python -u tools/bench_attn.py 16 1024 25 64 causal 0.0 >> gpurun_out/attn_swz/bench.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE --kernel-trace -d gpurun_out/attn_swz/s -o run -- python3 tools/bench_attn.py > gpurun_out/attn_swz/s.log 2>&1
rc=$?
cat gpurun_out/attn_swz/bench.log
python3 tools/pmc_db.py $(find gpurun_out/attn_swz/s -name "*.db" | head -1) > gpurun_out/attn_swz/s.txt 2>&1
find gpurun_out/attn_swz -name "*.db" -delete
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --kernel-trace -d gpurun_out/attn_swz/l -o run -- python3 tools/bench_attn.py 16 1024 25 64 causal 0.1 > gpurun_out/attn_swz/l.log 2>&1 || exit 1
python3 tools/pmc_db.py $(find gpurun_out/attn_swz/l -name "*.db" | head -1) attn > gpurun_out/attn_swz/l.txt 2>&1
find gpurun_out/attn_swz -name "*.db" -delete
timeout -k 10 600 python -u bench.py > gpurun_out/attn_swz/bench_step.json 2> gpurun_out/attn_swz/bench_step.err
rc=$?
tail -c 1500 gpurun_out/attn_swz/bench_step.json
exit $rc
