#!/bin/bash
# Keep words carried from a checkpoint's first forward to its recompute (ops/attention.py): numerics, the DM=1 vs
# DM=2 forward kernel times, then GPT-2-XL (checkpoint='always') with the reuse off / on, interleaved.
set -o pipefail
mkdir -p gpurun_out/keep
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu -k "attention or checkpoint or recompute" > gpurun_out/keep/tests.log 2>&1 || { tail -30 gpurun_out/keep/tests.log; exit 1; }
tail -1 gpurun_out/keep/tests.log
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/keep/dm -o run -- python3 tools/attn_long_dm_probe.py > gpurun_out/keep/dm.log 2>&1 || exit 1
python3 tools/kstats_db.py $(find gpurun_out/keep/dm -name "*.db" | head -1) attn_long
find gpurun_out/keep -name "*.db" -delete
for i in 1 2; do
  for arm in 0 1; do
    timeout -k 10 400 env MIPIPE_ATTN_KEEP_REUSE=$arm python -u bench.py --config gpt2_xl --steps 10 --warmup 3 --no-bubble > gpurun_out/keep/g_${arm}_$i.log 2>&1 || { tail -20 gpurun_out/keep/g_${arm}_$i.log; exit 1; }
    echo "reuse=$arm $i: $(grep -o '"value": [0-9.]*' gpurun_out/keep/g_${arm}_$i.log) $(grep -o '"gfxclk_mhz": {"mean": [0-9.]*' gpurun_out/keep/g_${arm}_$i.log) $(grep -o '"peak_hbm_gib_per_gpu": [^]]*]' gpurun_out/keep/g_${arm}_$i.log)"
  done
done
