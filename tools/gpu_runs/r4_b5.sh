#!/bin/bash
# IPC GPU tests with the inline default engine; GPT-2-XL A/B (defaults vs all round-4 GPT options off);
# PP=8 emulations with the balance objective on measured costs.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 MIPIPE_CALIB_DIR=$GRAFT_REPO_ROOT/gpurun_out/calib
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pipeline.py -k "ipc" > gpurun_out/ipc_tests5.log 2>&1 || { tail -30 gpurun_out/ipc_tests5.log; exit 1; }
tail -1 gpurun_out/ipc_tests5.log
val() { grep -o '"value": [0-9.]*' "$1" | head -1; }
for i in 1 2; do
  for arm in new old; do
    if [ $arm = old ]; then envs="MIPIPE_WGRAD_XT=0"; else envs=""; fi
    env $envs timeout -k 10 300 python -u bench.py --config gpt2_xl --steps 4 --warmup 2 --no-bubble > gpurun_out/gpt5_${arm}_$i.log 2>&1 || { tail -20 gpurun_out/gpt5_${arm}_$i.log; exit 1; }
    echo "gpt2_xl $arm run $i: $(val gpurun_out/gpt5_${arm}_$i.log)"
  done
done
for spec in "gpt2_xl measured balance always" "enc12_d4096 measured balance never" "enc12_d4096 analytic makespan never" "enc12_d4096 measured makespan never"; do
  set -- $spec
  timeout -k 10 500 python -u tools/pp_rank_emulation.py --config $1 --ranks all --steps 4 --plan $2 --objective $3 --checkpoint $4 > gpurun_out/emu5_$1_$2_$3_$4.log 2>&1 || { tail -20 gpurun_out/emu5_$1_$2_$3_$4.log; exit 1; }
  grep "^# plan\|^# per-rank\|^# slowest\|^# measured" gpurun_out/emu5_$1_$2_$3_$4.log
done
timeout -k 10 200 python -u tools/epilogue_cost_probe.py > gpurun_out/epilogue_probe.txt 2>&1; cat gpurun_out/epilogue_probe.txt
