#!/bin/bash
# attention_long.hip built with -amdgpu-mfma-vgpr-form: numerics, then kernel timing at GPT-2-XL's shape
# (B=18 S=1024 H=25 D=64 causal, p = 0.1), then the GPT-2-XL step.
set -o pipefail
mkdir -p gpurun_out/attn_vgpr
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu -k "attention" > gpurun_out/attn_vgpr/tests.log 2>&1 || { tail -30 gpurun_out/attn_vgpr/tests.log; exit 1; }
tail -1 gpurun_out/attn_vgpr/tests.log
timeout -k 10 120 python -u tools/bench_attn.py 18 1024 25 64 causal 0.1 2>&1 | tee gpurun_out/attn_vgpr/bench.log
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/attn_vgpr/k -o run -- python3 tools/bench_attn.py 18 1024 25 64 causal 0.1 > gpurun_out/attn_vgpr/k.log 2>&1 && \
python3 tools/kstats_db.py $(find gpurun_out/attn_vgpr/k -name "*.db" | head -1) attn_long > gpurun_out/attn_vgpr/k.txt 2>&1
find gpurun_out/attn_vgpr -name "*.db" -delete
cat gpurun_out/attn_vgpr/k.txt
timeout -k 10 400 python -u bench.py --config gpt2_xl --steps 10 --warmup 3 --no-bubble > gpurun_out/attn_vgpr/gpt.log 2>&1 || { tail -20 gpurun_out/attn_vgpr/gpt.log; exit 1; }
echo "gpt2_xl: $(grep -o '"value": [0-9.]*' gpurun_out/attn_vgpr/gpt.log) $(grep -o '"gfxclk_mhz": {[^}]*}' gpurun_out/attn_vgpr/gpt.log)"
