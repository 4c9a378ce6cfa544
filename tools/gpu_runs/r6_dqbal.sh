#!/bin/bash
# Long-sequence dQ with each wave on query rows w and 7 - w of its block (MIPIPE_ATTN_DQ_BAL=1) vs contiguous rows (0): numerics on the attention
# tests, kernel time at GPT-2-XL's shape, then the GPT-2-XL step; arms interleaved.
set -o pipefail
mkdir -p gpurun_out/dqbal
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
MIPIPE_ATTN_DQ_BAL=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu -k "attention" > gpurun_out/dqbal/tests.log 2>&1 || { tail -30 gpurun_out/dqbal/tests.log; exit 1; }
tail -1 gpurun_out/dqbal/tests.log
for i in 1 2; do
  for arm in 0 1; do
    MIPIPE_ATTN_DQ_BAL=$arm timeout -k 10 120 python -u tools/bench_attn.py 18 1024 25 64 causal 0.1 2>&1 | grep "kernels=1" | sed "s/^/dqbal=$arm $i /" || exit 1
  done
done
timeout -s KILL 120 env MIPIPE_ATTN_DQ_BAL=1 rocprofv3 --kernel-trace --stats -d gpurun_out/dqbal/k -o run -- python3 tools/bench_attn.py 18 1024 25 64 causal 0.1 > gpurun_out/dqbal/k.log 2>&1 || exit 1
python3 tools/kstats_db.py $(find gpurun_out/dqbal/k -name "*.db" | head -1) attn_long_dq
find gpurun_out/dqbal -name "*.db" -delete
for i in 1 2; do
  for arm in 0 1; do
    timeout -k 10 400 env MIPIPE_ATTN_DQ_BAL=$arm python -u bench.py --config gpt2_xl --steps 10 --warmup 3 --no-bubble > gpurun_out/dqbal/g_${arm}_$i.log 2>&1 || { tail -20 gpurun_out/dqbal/g_${arm}_$i.log; exit 1; }
    echo "dqbal=$arm $i gpt2_xl: $(grep -o '"value": [0-9.]*' gpurun_out/dqbal/g_${arm}_$i.log) $(grep -o '"gfxclk_mhz": {"mean": [0-9.]*' gpurun_out/dqbal/g_${arm}_$i.log)"
  done
done
