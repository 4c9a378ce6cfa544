#!/bin/bash
# Round 5: Pipe on the reference's structure, same box: stage streams shared vs dedicated, one partition, the engine;
# the overlap test alone; a kernel trace of the shared run.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > gpurun_out/pg3_$name.log 2>&1 || { tail -20 gpurun_out/pg3_$name.log; exit 1; }
  echo "$name: $(grep -o '"value": [0-9.]*' gpurun_out/pg3_$name.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/pg3_$name.log) $(grep -o '"gfxclk_mhz": {[^}]*}' gpurun_out/pg3_$name.log)"
}
R="--config ref_main --dtype fp32 --checkpoint never --steps 10 --warmup 3"
run shared --impl pipe --pipe-balance 8,8 --pipe-stage-streams shared $R
run dedicated --impl pipe --pipe-balance 8,8 --pipe-stage-streams dedicated $R
run one --impl pipe --pipe-balance 16 $R
run engine --chunks 4 --micro-batch 8 --no-bubble $R
run shared2 --impl pipe --pipe-balance 8,8 --pipe-stage-streams shared $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pipe_transport.py -k "overlap" > gpurun_out/overlap_test.log 2>&1; echo "overlap test rc=$?"; tail -3 gpurun_out/overlap_test.log
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --stats -d gpurun_out/pg3p -o run -- python3 bench.py --impl pipe --pipe-balance 8,8 --pipe-stage-streams shared $R --steps 3 --warmup 2 > gpurun_out/pg3p.log 2>&1 || { tail -5 gpurun_out/pg3p.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/pg3p/run_results.db 16 > gpurun_out/pg3p.txt 2>&1
head -20 gpurun_out/pg3p.txt | cut -c1-170
