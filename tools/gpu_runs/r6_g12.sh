#!/bin/bash
# GPT-2-XL: GELU backward as its own pass (default) vs folded into c_proj's dgrad epilogue with GELU' recomputed
# from the saved pre-activation (MIPIPE_FOLD_ACT=all) vs with GELU'(pre) saved by the forward
# (MIPIPE_FOLD_ACT=all MIPIPE_GELU_SAVE_GRAD=1).  Arms interleaved.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
run() {  # tag, env...
  local tag=$1; shift
  timeout -k 10 400 env "$@" python -u bench.py --config gpt2_xl --steps 10 --warmup 3 --no-bubble > gpurun_out/g12_$tag.log 2>&1 || { tail -20 gpurun_out/g12_$tag.log; return 1; }
  echo "$tag: $(grep -o '"value": [0-9.]*' gpurun_out/g12_$tag.log) $(grep -o '"gfxclk_mhz": {"mean": [0-9.]*' gpurun_out/g12_$tag.log)"
}
for i in 1 2; do
  run sep_$i MIPIPE_FOLD_ACT=auto || exit 1
  run fold_$i MIPIPE_FOLD_ACT=all || exit 1
  run foldsg_$i MIPIPE_FOLD_ACT=all MIPIPE_GELU_SAVE_GRAD=1 || exit 1
done
