#!/bin/bash
# Round 6: GPT-2-XL with GPT-2's MLP (no dropout after the GELU) -- the GELU backward then folds into c_proj's dgrad
# epilogue -- vs the torch-layer MLP (dropout 0.1 after the GELU, round 5's definition), and the folded backward with
# GELU'(pre) saved by the forward (MIPIPE_GELU_SAVE_GRAD=1) vs recomputed in the dgrad epilogue.  Arms interleaved.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
run() {  # tag, env..., -- bench args
  local tag=$1; shift
  local extra=""
  [[ $tag == old_* ]] && extra="--act-dropout 0.1"
  timeout -k 10 400 env "$@" python -u bench.py --config gpt2_xl --steps 10 --warmup 3 --no-bubble $extra > gpurun_out/g7_$tag.log 2>&1 || { tail -20 gpurun_out/g7_$tag.log; return 1; }
  echo "$tag: $(grep -o '"value": [0-9.]*' gpurun_out/g7_$tag.log) $(grep -o '"gfxclk_mhz": {"mean": [0-9.]*' gpurun_out/g7_$tag.log)"
}
for i in 1 2; do
  run old_$i MIPIPE_X=0 || exit 1
  run new_$i MIPIPE_GELU_SAVE_GRAD=0 || exit 1
  run newsg_$i MIPIPE_GELU_SAVE_GRAD=1 || exit 1
done
