#!/bin/bash
# LayerNorm wave-per-row forward: gamma / beta loaded with the row (MIPIPE_LN_ROWS_EARLY=1, new default) vs after the
# reductions (=0): per-call time at training shapes, bitwise outputs, then the GPT-2-XL step.  Arms interleaved.
set -o pipefail
mkdir -p gpurun_out/ln
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
for i in 1 2; do
  for arm in 0 1; do
    timeout -k 10 120 env MIPIPE_LN_ROWS_EARLY=$arm python -u tools/ln_fwd_ab.py "$GRAFT_REPO_ROOT" e${arm} 2>&1 | grep -E "1600|2048" || exit 1
  done
done
python tools/ln_fwd_ab.py --compare e0 e1 || exit 1
for i in 1 2; do
  for arm in 0 1; do
    timeout -k 10 400 env MIPIPE_LN_ROWS_EARLY=$arm python -u bench.py --config gpt2_xl --steps 10 --warmup 3 --no-bubble > gpurun_out/ln/g_${arm}_$i.log 2>&1 || { tail -20 gpurun_out/ln/g_${arm}_$i.log; exit 1; }
    echo "early=$arm $i: $(grep -o '"value": [0-9.]*' gpurun_out/ln/g_${arm}_$i.log) $(grep -o '"gfxclk_mhz": {"mean": [0-9.]*' gpurun_out/ln/g_${arm}_$i.log)"
  done
done
