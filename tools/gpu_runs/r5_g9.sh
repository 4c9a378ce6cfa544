#!/bin/bash
# Round 5: Pipe on the reference's structure (ref_main fp32, balance 8,8, one GPU): which part of the boundary
# machinery costs -- in-place hand-over vs copies, copy-stream count, hardware queues; plus the 4-wave GEMM PMC.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > gpurun_out/pg4_$name.log 2>&1 || { tail -20 gpurun_out/pg4_$name.log; exit 1; }
  echo "$name: $(grep -o '"value": [0-9.]*' gpurun_out/pg4_$name.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/pg4_$name.log)"
}
R="--impl pipe --pipe-balance 8,8 --config ref_main --dtype fp32 --checkpoint never --steps 10 --warmup 3"
run inplace_shared $R --pipe-boundary inplace --pipe-stage-streams shared
run inplace_dedicated $R --pipe-boundary inplace --pipe-stage-streams dedicated
run copy_shared_cs1 $R --pipe-boundary copy --pipe-stage-streams shared --pipe-copy-streams 1
run copy_dedicated_cs1 $R --pipe-boundary copy --pipe-stage-streams dedicated --pipe-copy-streams 1
run copy_shared $R --pipe-boundary copy --pipe-stage-streams shared
run inplace_shared_el --impl pipe --pipe-balance 8,8 --config ref_main --dtype fp32 --checkpoint except_last --steps 10 --warmup 3 --pipe-boundary inplace
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d gpurun_out/pmc5a -o p1 -- python3 tools/gemm_waves_pmc.py > gpurun_out/pmc5a.log 2>&1 || { tail -5 gpurun_out/pmc5a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum --kernel-trace -d gpurun_out/pmc5b -o p2 -- python3 tools/gemm_waves_pmc.py > gpurun_out/pmc5b.log 2>&1 || { tail -5 gpurun_out/pmc5b.log; exit 1; }
for d in pmc5a pmc5b; do python3 tools/pmc_db.py gpurun_out/$d/*.db gemm > gpurun_out/$d.txt 2>&1; done
cat gpurun_out/pmc5a.txt gpurun_out/pmc5b.txt | cut -c1-150 | head -80
rm -rf gpurun_out/pmc5a gpurun_out/pmc5b
