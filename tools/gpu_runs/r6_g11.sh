#!/bin/bash
# Round 6: GPT-2-XL weight gradients of qkv (4800 x 1600) / out / fc2 through the transposed GEMM (x transposed in
# the flush, bias gradient folded as a column sum of dY) instead of the I-contiguous GEMM + a separate column-sum
# pass over dY.  MIPIPE_WGRAD_XT_MIN_N: 6144 (default: fc1 only), 4800 (+ qkv), 1600 (every weight).  Interleaved.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
run() {  # tag, env...
  local tag=$1; shift
  timeout -k 10 400 env "$@" python -u bench.py --config gpt2_xl --steps 10 --warmup 3 --no-bubble > gpurun_out/g11_$tag.log 2>&1 || { tail -20 gpurun_out/g11_$tag.log; return 1; }
  echo "$tag: $(grep -o '"value": [0-9.]*' gpurun_out/g11_$tag.log) $(grep -o '"gfxclk_mhz": {"mean": [0-9.]*' gpurun_out/g11_$tag.log)"
}
for i in 1 2; do
  run base_$i MIPIPE_WGRAD_XT_MIN_N=6144 || exit 1
  run xt4800_$i MIPIPE_WGRAD_XT_MIN_N=4800 || exit 1
  run xt1600_$i MIPIPE_WGRAD_XT_MIN_N=1600 || exit 1
done
