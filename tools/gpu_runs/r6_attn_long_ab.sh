#!/bin/bash
# Same-box A/B of attention_long.hip with (B: the tree) and without (A: ab_tmp/A, MIPIPE_NO_FILE_FLAGS=1 build)
# -amdgpu-mfma-vgpr-form: kernel timing at GPT-2-XL's shape, then the GPT-2-XL step; arms interleaved.
set -o pipefail
mkdir -p gpurun_out/attn_ab
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
for i in 1 2; do
  for arm in A B; do
    d=$R; [ $arm = A ] && d=$R/ab_tmp/A
    (cd $d && timeout -k 10 120 python -u tools/bench_attn.py 18 1024 25 64 causal 0.1) > gpurun_out/attn_ab/k_${arm}_$i.log 2>&1 || { tail -5 gpurun_out/attn_ab/k_${arm}_$i.log; exit 1; }
    echo "$arm $i kernels: $(grep 'kernels=1' gpurun_out/attn_ab/k_${arm}_$i.log)"
  done
done
for i in 1 2; do
  for arm in A B; do
    d=$R; [ $arm = A ] && d=$R/ab_tmp/A
    (cd $d && timeout -k 10 400 python -u bench.py --config gpt2_xl --steps 10 --warmup 3 --no-bubble) > gpurun_out/attn_ab/g_${arm}_$i.log 2>&1 || { tail -20 gpurun_out/attn_ab/g_${arm}_$i.log; exit 1; }
    echo "$arm $i gpt2_xl: $(grep -o '"value": [0-9.]*' gpurun_out/attn_ab/g_${arm}_$i.log) $(grep -o '"gfxclk_mhz": {"mean": [0-9.]*' gpurun_out/attn_ab/g_${arm}_$i.log)"
  done
done
