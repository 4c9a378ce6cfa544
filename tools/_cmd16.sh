cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "attn_tests|300|python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k attention --timeout 120 --timeout-method thread" \
 "attn_p01|120|python tools/bench_attn.py 8 1024 25 64 causal 0.1" \
 "attn_p0|120|python tools/bench_attn.py 8 1024 25 64 causal 0.0" \
 "attn_p0_16row|120|env MIPIPE_ATTN_WIDE=0 python tools/bench_attn.py 8 1024 25 64 causal 0.0" \
 "gpt2|300|python bench.py --config gpt2_xl --steps 6 --warmup 2"
