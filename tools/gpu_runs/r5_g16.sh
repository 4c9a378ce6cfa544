#!/bin/bash
# Round 5: the bench's emulated plan pick -- plan tables (the pick vs every alternative) + a 2-rank shared-GPU smoke
# of bench.py's --plan-select emulate path.  usage: r5_g16.sh <config>:<pp>:<seconds> ...
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 MIPIPE_CALIB_DIR="$GRAFT_REPO_ROOT/gpurun_out/calib"
if [ "$SMOKE" = 1 ]; then
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --shared-gpu --plan measured --plan-select emulate --num-layers 4 --steps 2 --warmup 1 --no-bubble > gpurun_out/plan_select_smoke.log 2>&1 || { tail -30 gpurun_out/plan_select_smoke.log; exit 1; }
  grep -o '"plan_selection": {[^}]*' gpurun_out/plan_select_smoke.log | cut -c1-400
fi
for spec in "$@"; do
  IFS=: read c pp t <<< "$spec"
  timeout -k 10 $t python -u tools/plan_table.py --config "$c" --pp $pp --v 1,2,3,4 --steps 4 > gpurun_out/plan_table_${c}_pp$pp.txt 2>&1 || { tail -30 gpurun_out/plan_table_${c}_pp$pp.txt; exit 1; }
  grep -v "^wall\|^# PP=\|^## plan\|^   walls" gpurun_out/plan_table_${c}_pp$pp.txt | tail -20
done
