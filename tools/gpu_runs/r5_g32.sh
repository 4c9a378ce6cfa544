#!/bin/bash
# Round 5: the new enc12 default (micro-batch 128) -- the driver's command, the Pipe path, then the plan tables for the
# bench's PP=2 / PP=4 / PP=8 defaults at that micro-batch.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 MIPIPE_CALIB_DIR="$GRAFT_REPO_ROOT/gpurun_out/calib"
timeout -k 10 300 python -u bench.py > gpurun_out/mb128_default.log 2>&1 || { tail -20 gpurun_out/mb128_default.log; exit 1; }
echo "bench default: $(grep -o '"value": [0-9.]*' gpurun_out/mb128_default.log) $(grep -o '"micro_batch": [0-9]*' gpurun_out/mb128_default.log) $(grep -o '"peak_hbm_gib_per_gpu": \[[^]]*\]' gpurun_out/mb128_default.log)"
timeout -k 10 300 python -u bench.py --impl pipe --steps 10 --warmup 3 > gpurun_out/mb128_pipe.log 2>&1 || { tail -20 gpurun_out/mb128_pipe.log; exit 1; }
echo "pipe: $(grep -o '"value": [0-9.]*' gpurun_out/mb128_pipe.log) $(grep -o '"peak_hbm_gib_per_gpu": \[[^]]*\]' gpurun_out/mb128_pipe.log)"
for spec in enc12_d4096:2:300 enc12_d4096:4:360 enc12_d4096:8:420; do
  IFS=: read c pp t <<< "$spec"
  timeout -k 10 $t python -u tools/plan_table.py --config "$c" --pp $pp --v 1,2,3,4 --steps 3 > gpurun_out/plan_table_${c}_pp${pp}_mb128.txt 2>&1 || { tail -30 gpurun_out/plan_table_${c}_pp${pp}_mb128.txt; exit 1; }
  grep -E "bench default|^  +[0-9,]+ " gpurun_out/plan_table_${c}_pp${pp}_mb128.txt | head -6
done
