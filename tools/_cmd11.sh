cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "gpu_tests|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "smoke|300|python -u __graft_entry__.py smoke" \
 "bench|300|python bench.py --steps 10 --warmup 3" \
 "attn_gpt2_p01|120|python tools/bench_attn.py 8 1024 25 64 causal 0.1" \
 "attn_gpt2_p0|120|python tools/bench_attn.py 8 1024 25 64 causal 0.0" \
 "attn_enc_p0|120|python tools/bench_attn.py 32 128 16 256 nc 0.0"
